set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py tests/test_winograd_gpu.py > gpurun_out/c64_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6m abset:vodascheduler_amd.ops.conv3x3:USE_SPLIT_WGRAD_C64:resnet50-fp32:2
