set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py tests/test_ffn_gpu.py tests/test_layers_gpu.py > gpurun_out/t7v8_tests.log 2>&1 || { tail -30 gpurun_out/t7v8_tests.log; exit 1; }
tail -1 gpurun_out/t7v8_tests.log
timeout -k 10 300 python -u benchmarks/bench_splitgemm.py --quick --no-err --variants 8 --rounds 3 --out gpurun_out/t7v8_qkv.jsonl > gpurun_out/t7v8_probe.log 2>&1 || exit 1
bash benchmarks/gpu_lease.sh r6aa abset:vodascheduler_amd.ops.splitgemm:USE_T7_V8:bert-base-fp32:3
