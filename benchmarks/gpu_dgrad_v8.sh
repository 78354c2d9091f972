set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/dg8_tests.log 2>&1 || { tail -30 gpurun_out/dg8_tests.log; exit 1; }
tail -1 gpurun_out/dg8_tests.log
bash benchmarks/gpu_lease.sh r6x abset:vodascheduler_amd.ops.conv3x3:USE_SPLIT_CONV_DGRAD:resnet50-fp32:3
