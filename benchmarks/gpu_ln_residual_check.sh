#!/bin/bash
# GPU check of the residual add fused into the LayerNorm kernel: numerics, then the BERT-base
# step with and without the fusion (VODA_LN_RESIDUAL, alternating, same box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ln_res_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  VODA_LN_RESIDUAL=$v timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 >> gpurun_out/bert_lnres_v$v.log 2>&1 || exit $?
done
