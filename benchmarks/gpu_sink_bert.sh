#!/bin/bash
# GPU check of the residual-stream gradient hand-off in the transformer layers: numerics,
# then the BERT-base step with and without it (alternating, same box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_wgrad.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sink_bert_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  VODA_GRAD_SINK=$v timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 >> gpurun_out/bert_sink_v$v.log 2>&1 || exit $?
done
