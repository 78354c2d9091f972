set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py tests/test_ffn_gpu.py tests/test_layers_gpu.py > gpurun_out/v8f_tests.log 2>&1 || { tail -30 gpurun_out/v8f_tests.log; exit 1; }
tail -1 gpurun_out/v8f_tests.log
bash benchmarks/gpu_lease.sh r6u abset:vodascheduler_amd.ops.splitgemm:USE_V8_FWD:bert-base-fp32:3
