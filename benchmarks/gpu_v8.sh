set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py tests/test_ffn_gpu.py tests/test_layers_gpu.py > gpurun_out/v8_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6s abset:vodascheduler_amd.ops.splitgemm:USE_V8_KMAJOR_B:bert-base-fp32:3
