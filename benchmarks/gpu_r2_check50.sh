#!/bin/bash
# Round-2 check 50: LayerNorm backward dgamma/dbeta as fp32 atomic adds into the flat gradient
# (no col_sum launch; VODA_LN_ATOMIC=0 = partial rows + col_sum): numerics, BERT-base A/B.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c50
mkdir -p $O
true
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    VODA_LN_ATOMIC=$v timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 | sed "s/^{/{\"env\": \"VODA_LN_ATOMIC=$v\", /" >> $O/ab_ln_atomic.jsonl || exit 4
  done
done
cut -c1-120 $O/ab_ln_atomic.jsonl
