#!/bin/bash
# Round-2 check 46: attention fwd / dQ with register-prefetched K/V tiles (next tile's global
# loads in flight during this tile's compute): numerics, micro-benchmark, BERT kernel times.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c46
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_attention_gpu.py tests/test_layers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -u benchmarks/bench_attention.py > $O/attn_micro.txt 2>&1 || { tail -5 $O/attn_micro.txt; exit 3; }
tail -1 $O/attn_micro.txt
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bert -o bert -- python3 $R/benchmarks/model_step.py --model bert-base --batch 64 --steps 10 --warmup 6 --profile-marker ) > $O/prof_bert.log 2>&1 || { tail -10 $O/prof_bert.log; exit 6; }
mkdir -p $O/prof_bert
python3 $R/benchmarks/trace_window_stats.py /tmp/prof_bert/bert_kernel_trace.csv $O/prof_bert/steady_kernel_stats.csv >> $O/prof_bert.log 2>&1 || exit 7
tail -1 $O/prof_bert.log
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_bert/steady_kernel_stats.csv')):
    if 'attn' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,2), r['Name'][:70])
"
for rep in 1 2; do
  timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 >> $O/steps.jsonl || exit 4
done
cut -c1-100 $O/steps.jsonl
