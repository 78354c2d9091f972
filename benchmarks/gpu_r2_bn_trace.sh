#!/bin/bash
# Per-dispatch BN kernel durations over the ResNet-50 shapes (kernel trace only), per
# reduction-pass tuning (deep,blocks,sweep).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/bnt
for t in ${TUNINGS:-1,1024,0 1,512,0}; do
  n=${t//,/_}
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/bnt_$n -o bnt -- python3 $R/benchmarks/bench_bn_passes.py --iters 5 --tuning $t ) > $R/gpurun_out/bnt/run_$n.log 2>&1 || { tail -5 $R/gpurun_out/bnt/run_$n.log; exit 3; }
  f=$(find /tmp/bnt_$n -name "*kernel_trace.csv" | head -1); cp $f $R/gpurun_out/bnt/trace_$n.csv
done
echo done
