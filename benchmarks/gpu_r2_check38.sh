#!/bin/bash
# Round-2 check 38: attention mask codes staged in LDS per key tile (fwd + dQ passes):
# numerics, attention micro-benchmark, BERT-base / NMT step.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c38
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -u benchmarks/bench_attention.py > $O/attn_micro.txt 2>&1 || { tail -5 $O/attn_micro.txt; exit 3; }
tail -8 $O/attn_micro.txt
for rep in 1 2; do
  timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 >> $O/steps.jsonl || exit 4
  timeout -k 10 200 python3 -u benchmarks/model_step.py --model transformer --steps 30 --warmup 5 >> $O/steps.jsonl || exit 5
done
cat $O/steps.jsonl
