set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py > gpurun_out/w1p_tests.log 2>&1 && \
timeout -k 10 300 python -u benchmarks/bench_winograd.py > gpurun_out/w1p_bench.jsonl 2> gpurun_out/w1p_bench.err && \
bash benchmarks/gpu_lease.sh r6k abset:vodascheduler_amd.ops.winograd:ONEPOS:resnet50-fp32:2
