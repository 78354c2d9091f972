#!/bin/bash
# Round-2 check 47: attention workgroup size cap (VODA_ATTN_MAXW=1/2/4: more, smaller
# workgroups per (batch, head)): numerics at each cap, micro-benchmark, BERT-base step A/B.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c47
mkdir -p $O
for w in 1 2; do
  VODA_ATTN_MAXW=$w timeout -k 10 300 python3 -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_w$w.log 2>&1 || { tail -30 $O/tests_w$w.log; exit 2; }
  tail -1 $O/tests_w$w.log
done
for w in 4 2 1; do
  VODA_ATTN_MAXW=$w timeout -k 10 200 python3 -u benchmarks/bench_attention.py > $O/attn_micro_w$w.txt 2>&1 || { tail -5 $O/attn_micro_w$w.txt; exit 3; }
  echo "maxw $w $(tail -1 $O/attn_micro_w$w.txt)"
done
for rep in 1 2; do
  for w in 4 2 1; do
    VODA_ATTN_MAXW=$w timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 | sed "s/^{/{\"env\": \"VODA_ATTN_MAXW=$w\", /" >> $O/ab_maxw.jsonl || exit 4
  done
done
cut -c1-130 $O/ab_maxw.jsonl
