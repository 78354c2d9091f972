set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py tests/test_ffn_gpu.py > gpurun_out/t7b_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6g abset:vodascheduler_amd.ops.splitgemm:USE_T7:bert-base-fp32:2
