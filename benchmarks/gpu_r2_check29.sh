#!/bin/bash
# Round-2 check 29: does a stock-autograd (fold-hook) gradient survive repeated graph replays?
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c29
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest tests/test_stepgraph_fold_gpu.py -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|replay|assert" $O/pytest.log | head -30
exit $rc
