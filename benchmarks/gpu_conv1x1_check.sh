#!/bin/bash
# 1x1-conv GEMM path: numerics, ResNet-50 step A/B, full GPU suite, N=1 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/conv1x1_tests.log 2>&1 || exit $?
VODA_CONV1X1_GEMM=1 timeout -k 10 300 python -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/resnet_gemm_on.log 2>&1 || exit $?
VODA_CONV1X1_GEMM=0 timeout -k 10 300 python -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/resnet_gemm_off.log 2>&1 || exit $?
VODA_CONV1X1_GEMM=1 timeout -k 10 300 python -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/resnet_gemm_on2.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --out gpurun_out/bench_n1.json > gpurun_out/bench_n1.log 2>&1 || exit $?
