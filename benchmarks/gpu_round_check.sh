#!/bin/bash
# Round-end style GPU check: the whole GPU test suite, smoke(), then bench.py at N=1.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --out gpurun_out/bench_n1.json > gpurun_out/bench_n1.log 2>&1 || exit $?
