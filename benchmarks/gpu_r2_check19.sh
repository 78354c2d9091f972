#!/bin/bash
# Round-2 check 19: full GPU suite + smoke + N=1 bench with detail after the wgrad choice /
# attention LDS / cross-attention changes.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c19
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/c19/pytest_gpu.log 2>&1 || { tail -40 $R/gpurun_out/c19/pytest_gpu.log; exit 2; }
tail -2 $R/gpurun_out/c19/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/gpurun_out/c19/smoke.log 2>&1 || { tail -20 $R/gpurun_out/c19/smoke.log; exit 3; }
tail -1 $R/gpurun_out/c19/smoke.log
timeout -k 10 600 python3 bench.py --out $R/gpurun_out/c19/bench_n1_detail.json > $R/gpurun_out/c19/bench.log 2>&1 || { tail -20 $R/gpurun_out/c19/bench.log; exit 4; }
tail -1 $R/gpurun_out/c19/bench.log
echo done
