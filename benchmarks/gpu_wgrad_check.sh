#!/bin/bash
# GPU check of the split-K wgrad kernel: numerics, microbenchmark, BERT-base step A/B,
# and the hipBLASLt path tuned by PyTorch TunableOp for comparison.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wgrad.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wgrad_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/bench_wgrad.py > gpurun_out/bench_wgrad.log 2>&1 || exit $?
VODA_WGRAD=1 timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 > gpurun_out/bert_wgrad_on.log 2>&1 || exit $?
VODA_WGRAD=0 timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 > gpurun_out/bert_wgrad_off.log 2>&1 || exit $?
VODA_WGRAD_VARIANT=0 timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 > gpurun_out/bert_wgrad_v0.log 2>&1 || exit $?
