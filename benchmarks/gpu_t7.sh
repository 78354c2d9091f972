# 128 x 96 split-GEMM tile: numerics, then the BERT-shape sweep with it
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/t7_tests.log 2>&1 && \
timeout -k 10 700 python -u benchmarks/bench_splitgemm.py --no-err --rounds 3 --reps 10 --out gpurun_out/t7_sweep.jsonl > gpurun_out/t7_sweep.log 2>&1
