# Winograd SX2 (64 output channels / workgroup): numerics, per-layer timing
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py > gpurun_out/wino2_tests.log 2>&1 && \
timeout -k 10 300 python -u benchmarks/bench_winograd.py > gpurun_out/wino2_bench.jsonl 2> gpurun_out/wino2_bench.err
