set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py tests/test_conv1x1_f32_gpu.py > gpurun_out/v8c_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6t abset:vodascheduler_amd.ops.splitgemm:CONV_WGRAD_V8:resnet50-fp32:2 abset:vodascheduler_amd.ops.conv1x1:WGRAD_V8:resnet50-fp32:2
