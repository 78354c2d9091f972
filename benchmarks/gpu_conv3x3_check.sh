#!/bin/bash
# GPU check of the implicit-GEMM 3x3 weight-gradient kernel: numerics, then the ResNet-50
# bs256 step with and without it (alternating, same box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv3x3.py tests/test_conv1x1.py tests/test_wgrad.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/conv3_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  VODA_CONV_WGRAD=$v timeout -k 10 300 python -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 >> gpurun_out/resnet_conv3_v$v.log 2>&1 || exit $?
done
