#!/bin/bash
# Round-2 check 52: large-head-dim attention (NMT D = 256, T = 20) with the row-operand
# fragments loaded from global instead of LDS images (LDS per one-wave workgroup 37-54 KB ->
# ~20 KB, so more workgroups per CU): numerics, NMT kernel times, NMT / BERT steps.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c52
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_attention_gpu.py tests/test_layers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_nmt -o nmt -- python3 $R/benchmarks/model_step.py --model transformer --batch 512 --steps 10 --warmup 6 --profile-marker ) > $O/prof_nmt.log 2>&1 || { tail -10 $O/prof_nmt.log; exit 6; }
mkdir -p $O/prof_nmt
python3 $R/benchmarks/trace_window_stats.py /tmp/prof_nmt/nmt_kernel_trace.csv $O/prof_nmt/steady_kernel_stats.csv >> $O/prof_nmt.log 2>&1 || exit 7
tail -1 $O/prof_nmt.log
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_nmt/steady_kernel_stats.csv')):
    if 'attn' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,2), r['Name'][:80])
"
for rep in 1 2; do
  timeout -k 10 200 python3 -u benchmarks/model_step.py --model transformer --steps 30 --warmup 5 >> $O/steps.jsonl || exit 4
  timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 >> $O/steps.jsonl || exit 5
done
cut -c1-100 $O/steps.jsonl
