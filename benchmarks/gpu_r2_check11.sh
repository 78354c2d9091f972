#!/bin/bash
# Round-2 check 11: bisect the ResNet-50 hipGraph replay failure (non-finite layer1 conv3
# weight gradients from the second real-update replay on) over the model's fused paths.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c11
for env in "VODA_NONE=1" "VODA_GRAD_SINK=0" "VODA_CONV1X1_GEMM=0" "VODA_CONV_WGRAD=0" "VODA_FUSED_BN=0"; do
  env $env timeout -k 10 200 python3 benchmarks/graph_diag.py --model resnet50 --batch 64 --nan-probe 4 --graph-only > $R/gpurun_out/c11/probe_${env%%=*}.json 2> $R/gpurun_out/c11/probe.err || { tail -5 $R/gpurun_out/c11/probe.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$R/gpurun_out/c11/probe_${env%%=*}.json'))
print('$env', [(r['step'], round(r['loss'],3), r['n_bad_grads'], r['bad_grads'][:3]) for r in d['probe_graph']['rows']])
"
done
echo done
