set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv1x1_f32_gpu.py tests/test_resnet_glue_gpu.py > gpurun_out/f1_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6q abset:vodascheduler_amd.ops.conv1x1:USE_SPLIT_FWD_F32:resnet50-fp32:2
