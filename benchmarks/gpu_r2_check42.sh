#!/bin/bash
# Round-2 check 42: LayerNorm kernels with the per-row statistics (backward) and gamma/beta
# (forward) loads issued with the row data: numerics, BERT-base kernel times, steps.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c42
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py tests/test_layers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bert -o bert -- python3 $R/benchmarks/model_step.py --model bert-base --batch 64 --steps 10 --warmup 6 --profile-marker ) > $O/prof_bert.log 2>&1 || { tail -10 $O/prof_bert.log; exit 6; }
mkdir -p $O/prof_bert
python3 $R/benchmarks/trace_window_stats.py /tmp/prof_bert/bert_kernel_trace.csv $O/prof_bert/steady_kernel_stats.csv >> $O/prof_bert.log 2>&1 || exit 7
tail -1 $O/prof_bert.log
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_bert/steady_kernel_stats.csv')):
    if 'ln_' in r['Name'] or 'attn' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,2), r['Name'][:70])
"
for rep in 1 2; do
  timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 >> $O/steps.jsonl || exit 4
  timeout -k 10 200 python3 -u benchmarks/model_step.py --model transformer --steps 30 --warmup 5 >> $O/steps.jsonl || exit 5
done
cut -c1-100 $O/steps.jsonl
