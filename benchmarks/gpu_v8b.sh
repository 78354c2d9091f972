set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/v8b_tests.log 2>&1 || { tail -30 gpurun_out/v8b_tests.log; exit 1; }
timeout -k 10 500 python -u benchmarks/bench_splitgemm.py --variants 8 --variant-splits --no-sweep --no-err --split-list 1,2,3,4,5,6,7,8,10,12,16,21 --out gpurun_out/v8_split_sweep.jsonl > gpurun_out/v8sweep.log 2>&1 || { tail -20 gpurun_out/v8sweep.log; exit 1; }
bash benchmarks/gpu_lease.sh r6v abset:vodascheduler_amd.ops.conv1x1:USE_SPLIT_FWD_F32:resnet50-fp32:2 abset:vodascheduler_amd.ops.conv1x1:USE_SPLIT_GEMM_F32:resnet50-fp32:2 abset:vodascheduler_amd.ops.splitgemm:CONV_FWD_V8:resnet50-fp32:2
