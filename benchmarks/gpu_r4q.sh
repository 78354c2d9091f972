# GPU test suite, smoke, then a 2-rank elastic rehearsal sharing the one GPU (gloo data plane,
# fp32 default): live resizes through the real worker pool on real kernels.
set -o pipefail
OUT=gpurun_out/r4q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 4 --warmup 2 --jobs 12 --share-gpu --comm-backend gloo --control FIFO --deadline 500 \
  > $OUT/share2.json 2> $OUT/share2.err || { tail -30 $OUT/share2.err; exit 1; }
tail -c 1500 $OUT/share2.json
