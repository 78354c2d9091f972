#!/bin/bash
# Round-2 check 54: fold low-precision autograd gradients into the fp32 flat buffer with a cast
# + same-dtype add instead of PyTorch's mixed-dtype add (VODA_FOLD_CAST): ResNet-50 step A/B
# and the elementwise kernels of each variant (rocprofv3).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c54
mkdir -p $O
for rep in 1 2; do
  for v in 0 1; do
    VODA_FOLD_CAST=$v timeout -k 10 300 python3 -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 | sed "s/^{/{\"env\": \"VODA_FOLD_CAST=$v\", /" >> $O/ab_fold.jsonl || exit 4
  done
done
cut -c1-120 $O/ab_fold.jsonl
for v in 0 1; do
  ( cd /tmp && VODA_FOLD_CAST=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r$v -o r -- python3 $R/benchmarks/model_step.py --model resnet50 --batch 256 --steps 10 --warmup 6 --profile-marker ) > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 6; }
  mkdir -p $O/prof_$v
  python3 $R/benchmarks/trace_window_stats.py /tmp/prof_r$v/r_kernel_trace.csv $O/prof_$v/steady_kernel_stats.csv >> $O/prof_$v.log 2>&1 || exit 7
  echo "FOLD_CAST=$v $(tail -1 $O/prof_$v.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$v/steady_kernel_stats.csv')):
    n=r['Name']
    if 'at::native' in n and ('add' in n or 'copy' in n): print('  ', r['Calls'], round(float(r['AverageNs'])/1e3,1), n[:90])
"
done
