# Winograd SX2 (64 output channels / workgroup): numerics, per-layer timing, then the 1x1 split probe
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py > gpurun_out/wino2_tests.log 2>&1 && \
timeout -k 10 300 python -u benchmarks/bench_winograd.py > gpurun_out/wino2_bench.jsonl 2> gpurun_out/wino2_bench.err && \
timeout -k 10 500 python -u benchmarks/bench_resnet_1x1_split.py --out gpurun_out/r1x1.jsonl > gpurun_out/r1x1.log 2>&1
