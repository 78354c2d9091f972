set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py tests/test_ffn_gpu.py tests/test_layers_gpu.py > gpurun_out/rs_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6l abset:vodascheduler_amd.ops.splitgemm:USE_FUSED_ROW_SUMS:bert-base-fp32:2
