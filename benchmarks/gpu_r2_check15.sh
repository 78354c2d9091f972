#!/bin/bash
# Round-2 check 15 (eager only, no graph replay): do the NMT step's kernels write every
# output element?  Attention outputs pre-filled with NaN; whole NMT step on a NaN-poisoned
# allocator.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c15
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py -k "writes_every" > $R/gpurun_out/c15/pytest.log 2>&1; echo "pytest rc=$?"; tail -15 $R/gpurun_out/c15/pytest.log
timeout -k 10 150 python3 benchmarks/graph_diag.py --model transformer --batch 64 --nan-probe 3 --poison > $R/gpurun_out/c15/nmt_poison.json 2> $R/gpurun_out/c15/nmt_poison.err || { tail -5 $R/gpurun_out/c15/nmt_poison.err; exit 3; }
python3 -c "
import json; d=json.load(open('$R/gpurun_out/c15/nmt_poison.json'))
for r in d['probe_eager_poisoned']['rows']: print('  ', r['step'], round(r['loss'],4), r['n_bad_grads'], r['bad_grads'][:6])
"
echo done
