# thin (64 x 256 / 256 x 64) split-GEMM tiles: numerics, then the ResNet-50 fp32 step A/B
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/thin_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6e abset:vodascheduler_amd.ops.conv1x1:USE_THIN_TILES:resnet50-fp32:2
