#!/bin/bash
# Round-2 check 33: compile-time-window (3x3/2) maxpool and fused stem kernels with all window
# loads in flight: numerics, per-kernel times (rocprofv3), ResNet-50 A/B with the fused stem
# on/off; torch-profiler op table of ResNet-50 (which aten ops launch the remaining
# elementwise kernels); steady-state BERT-base kernel profile after the fused cross-entropy.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c33
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_batchnorm_gpu.py -m gpu -x -q -k "maxpool" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
export VODA_FUSED_BN_POOL=1
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_stem -o stem -- python3 $R/benchmarks/bench_stem.py --only-bn-pool ) > $O/prof_stem.log 2>&1 || { tail -20 $O/prof_stem.log; exit 3; }
grep stem_bn $O/prof_stem.log
find /tmp/prof_stem -name "*kernel_stats.csv" -exec cp {} $O/stem_kernel_stats.csv \;
python3 -c "
import csv
rows=list(csv.DictReader(open('$O/stem_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:110])
"
unset VODA_FUSED_BN_POOL
for rep in 1 2; do
  for v in 0 1; do
    VODA_FUSED_BN_POOL=$v timeout -k 10 300 python3 -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 | sed "s/^{/{\"env\": \"VODA_FUSED_BN_POOL=$v\", /" >> $O/ab_pool.jsonl || exit 4
  done
done
cat $O/ab_pool.jsonl
timeout -k 10 300 python3 -u benchmarks/model_step.py --model resnet50 --steps 10 --warmup 5 --torch-profile $O/torch_ops_resnet50.txt > $O/tp.log 2>&1 || { tail -5 $O/tp.log; exit 5; }
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bert -o bert -- python3 $R/benchmarks/model_step.py --model bert-base --batch 64 --steps 10 --warmup 6 --profile-marker ) > $O/prof_bert.log 2>&1 || { tail -10 $O/prof_bert.log; exit 6; }
mkdir -p $O/prof_bert
python3 $R/benchmarks/trace_window_stats.py /tmp/prof_bert/bert_kernel_trace.csv $O/prof_bert/steady_kernel_stats.csv >> $O/prof_bert.log 2>&1 || exit 7
tail -3 $O/prof_bert.log
echo done
