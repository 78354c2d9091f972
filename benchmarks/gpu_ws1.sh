# wave-specialised split GEMM: numerics, BERT-shape probe, PMC of the fc1 forward (variants 0 / 6 / 7)
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/ws_tests.log 2>&1 && \
timeout -k 10 400 python -u benchmarks/bench_splitgemm.py --no-sweep --no-err --variants 7 --variant-splits --rounds 3 --reps 10 --out gpurun_out/ws_probe3.jsonl > gpurun_out/ws_probe3.log 2>&1 && \
PMC_OUT=pmc_ws3 SG_ARGS="--shape 8192,3072,768 --op fwd --variants 0,6,7" bash benchmarks/pmc_splitgemm.sh
