#!/bin/bash
# Round-4 A/B: fp32 stage-4 1x1 weight gradients on hipBLASLt (beta = 1 into the flat gradient)
# vs MIOpen's igemm_wrw + fold-in add, ResNet-50 fp32 step, interleaved on one box.
set -o pipefail
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv1x1.py tests/test_conv1x1_f32_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in 1 0; do
    VODA_BLAS_WGRAD_F32=$v timeout -k 10 240 python -u benchmarks/model_step.py --model resnet50 --precision fp32 --steps 30 --warmup 10 > $O/run_${v}_$i.log 2>&1 || { tail -20 $O/run_${v}_$i.log; exit 1; }
    echo "blas_wgrad=$v rep=$i $(grep '^{' $O/run_${v}_$i.log | tail -1 | cut -c1-160)"
  done
done
