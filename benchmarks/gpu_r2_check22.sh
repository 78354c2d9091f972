#!/bin/bash
# Round-2 check 22: LayerNorm backward grid cap A/B on the BERT-base step (+ LN tests at 1024).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c22
VODA_LN_BWD_BLOCKS=1024 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "layernorm or layer_norm or ln_" > $R/gpurun_out/c22/pytest_ln.log 2>&1 || { tail -30 $R/gpurun_out/c22/pytest_ln.log; exit 2; }
tail -2 $R/gpurun_out/c22/pytest_ln.log
for rep in 1 2; do
  for b in 256 512 1024 2048; do
    VODA_LN_BWD_BLOCKS=$b timeout -k 10 240 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 40 --warmup 6 | sed "s/^{/{\"ln_bwd_blocks\": $b, /" >> $R/gpurun_out/c22/ab_ln.jsonl || exit 4
  done
done
cat $R/gpurun_out/c22/ab_ln.jsonl
echo done
