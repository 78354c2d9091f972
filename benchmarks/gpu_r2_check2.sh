#!/bin/bash
# Round-2 check 2: GPU tests touched since check 1, overlapped-optimizer A/B, bench N=1.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_conv1x1.py tests/test_conv3x3.py tests/test_wgrad.py \
  tests/test_layers_gpu.py tests/test_runtime_gpu.py tests/test_stepgraph_gpu.py tests/test_batchnorm_gpu.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2c2_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r2c2_pytest.log
tail -12 gpurun_out/r2c2_pytest.log
for rep in 1 2; do
  for ov in "" "--overlap-opt"; do
    timeout -k 10 240 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 30 --warmup 6 $ov >> gpurun_out/r2c2_ab_overlap.jsonl || exit 2
    timeout -k 10 240 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 20 --warmup 6 $ov >> gpurun_out/r2c2_ab_overlap.jsonl || exit 2
  done
done
cat gpurun_out/r2c2_ab_overlap.jsonl
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2c2_bench_n1.json 2> gpurun_out/r2c2_bench_n1.err || { tail -20 gpurun_out/r2c2_bench_n1.err; exit 3; }
cat gpurun_out/r2c2_bench_n1.json
