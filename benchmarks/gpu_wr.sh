set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py -k conv_wgrad > gpurun_out/wr_tests.log 2>&1 || { tail -30 gpurun_out/wr_tests.log; exit 1; }
tail -1 gpurun_out/wr_tests.log
bash benchmarks/gpu_lease.sh r6y abset:vodascheduler_amd.ops.splitgemm:CONV_WGRAD_V8_ROUNDS:resnet50-fp32:3
