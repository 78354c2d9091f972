#!/bin/bash
# Round-2 first GPU check: full GPU test suite, 1-GPU bench, 2-rank gloo rehearsal on one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r2c1_pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r2c1_pytest_gpu.log
tail -3 gpurun_out/r2c1_pytest_gpu.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r2c1_bench_n1_full.json \
  > gpurun_out/r2c1_bench_n1.json 2> gpurun_out/r2c1_bench_n1.err || { echo "bench n1 failed"; tail -20 gpurun_out/r2c1_bench_n1.err; exit 1; }
cat gpurun_out/r2c1_bench_n1.json
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --share-gpu --comm-backend gloo --steps 4 --warmup 2 --jobs 8 \
  > gpurun_out/r2c1_bench_share2.json 2> gpurun_out/r2c1_bench_share2.err || { echo "share2 failed"; tail -20 gpurun_out/r2c1_bench_share2.err; exit 1; }
cat gpurun_out/r2c1_bench_share2.json
