#!/bin/bash
# GPU A/B of the LayerNorm gradient accumulation (VODA_LN_DIRECT), alternating, same box.
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 0 1; do
  VODA_LN_DIRECT=$v timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 >> gpurun_out/bert_ln_v$v.log 2>&1 || exit $?
done
