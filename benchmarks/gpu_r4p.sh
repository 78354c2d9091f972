# Round-end style checks: the driver's exact bench command (fp32 default, shipped TunableOp
# results), then the GPU test suite and smoke.
set -o pipefail
OUT=gpurun_out/${R4P_OUT:-r4p}
mkdir -p $OUT
start=$(date +%s)
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
echo "driver bench wall $(( $(date +%s) - start )) s" | tee $OUT/bench_time.txt
tail -c 600 $OUT/bench.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
