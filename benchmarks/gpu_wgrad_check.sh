#!/bin/bash
# GPU check of the split-K wgrad kernel variants: numerics, microbenchmark, BERT-base step A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wgrad.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wgrad_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u benchmarks/bench_wgrad.py ${WGRAD_BENCH_ARGS:-} > gpurun_out/bench_wgrad.log 2>&1 || exit $?
for v in ${WGRAD_STEP_VARIANTS:-2 6 7 8}; do
  VODA_WGRAD_VARIANT=$v timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 > gpurun_out/bert_wgrad_v$v.log 2>&1 || exit $?
done
