# stride-2 3x3 input gradients as polyphase implicit GEMMs: numerics, ResNet-50 fp32 step A/B
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/s2_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6j abset:vodascheduler_amd.ops.conv3x3:USE_SPLIT_CONV_DGRAD:resnet50-fp32:2
