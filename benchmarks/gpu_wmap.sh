set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/wm_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6o abset:vodascheduler_amd.ops.splitgemm:WRITE_MAP:bert-base-fp32:2 abset:vodascheduler_amd.ops.splitgemm:WRITE_MAP:resnet50-fp32:2
