#!/bin/bash
# Per-dispatch BN apply-pass durations per apply-grid setting (env), kernel trace only.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/bna
i=0
for e in "VODA_BN_APPLY_ITERS=4" "VODA_BN_APPLY_ITERS=2" "VODA_BN_APPLY_ITERS=8" "VODA_BN_APPLY_ITERS=16" "VODA_BN_APPLY_CAP=1024 VODA_BN_APPLY_ITERS=1000000" "VODA_BN_APPLY_CAP=2048 VODA_BN_APPLY_ITERS=1000000"; do
  i=$((i+1))
  ( cd /tmp && env $e timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/bna_$i -o bna -- python3 $R/benchmarks/bench_bn_passes.py --iters 5 ) > $R/gpurun_out/bna/run_$i.log 2>&1 || { tail -5 $R/gpurun_out/bna/run_$i.log; exit 3; }
  f=$(find /tmp/bna_$i -name "*kernel_trace.csv" | head -1); cp $f "$R/gpurun_out/bna/trace_${i}_${e// /_}.csv"
done
echo done
