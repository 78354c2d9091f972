set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py -k "wave_specialised" > gpurun_out/v8_tests.log 2>&1 && \
timeout -k 10 600 python -u benchmarks/bench_splitgemm.py --no-sweep --no-err --variants 8 --variant-splits --rounds 3 --reps 10 --out gpurun_out/v8_probe.jsonl > gpurun_out/v8_probe.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6r tests smoke bench-fp32
