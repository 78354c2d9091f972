#!/bin/bash
# GPU check of the residual-gradient hand-off (ops/conv1x1.GradSink): numerics, then the
# ResNet-50 bs256 step with and without it (same box, one process each), then a steady-state
# kernel profile with it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1.py tests/test_batchnorm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sink_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  VODA_GRAD_SINK=$v timeout -k 10 300 python -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 >> gpurun_out/resnet_sink_v$v.log 2>&1 || exit $?
done
