#!/bin/bash
# Round-2 check 8: BN tests after the flat-path removal; per-convolution hipGraph replay probe
# (MIOpen vs GEMM path) to pin the ResNet-50 replay failure to one library call.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c8
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batchnorm_gpu.py > $R/gpurun_out/c8/pytest_bn.log 2>&1 || { tail -30 $R/gpurun_out/c8/pytest_bn.log; exit 2; }
tail -2 $R/gpurun_out/c8/pytest_bn.log
timeout -k 10 500 python3 benchmarks/graph_conv_probe.py --steps 6 > $R/gpurun_out/c8/conv_probe.jsonl 2> $R/gpurun_out/c8/conv_probe.err || { tail -5 $R/gpurun_out/c8/conv_probe.err; exit 3; }
python3 -c "
import json
for l in open('$R/gpurun_out/c8/conv_probe.jsonl'):
    d=json.loads(l); print(d['case'], d['path'], 'first_bad', d['first_bad_step'], [(r['grad_finite'], '%.2g'%r['grad_rel'], '%.2g'%r['weight_rel']) for r in d['rows']])
"
echo done
