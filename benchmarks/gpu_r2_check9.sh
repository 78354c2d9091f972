#!/bin/bash
# Round-2 check 9: do library backward kernels read their uninitialised outputs?  Eager steps
# right after the caching allocator was filled with NaN: per convolution, and the whole
# ResNet-50 step.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c9
timeout -k 10 300 python3 benchmarks/graph_conv_probe.py --poison > $R/gpurun_out/c9/conv_poison.jsonl 2> $R/gpurun_out/c9/conv_poison.err || { tail -5 $R/gpurun_out/c9/conv_poison.err; exit 3; }
cat $R/gpurun_out/c9/conv_poison.jsonl
timeout -k 10 300 python3 benchmarks/graph_diag.py --model resnet50 --batch 64 --nan-probe 4 --poison > $R/gpurun_out/c9/resnet50_poison.json 2> $R/gpurun_out/c9/resnet50_poison.err || { tail -5 $R/gpurun_out/c9/resnet50_poison.err; exit 4; }
python3 -c "
import json; d=json.load(open('$R/gpurun_out/c9/resnet50_poison.json'))
for r in d['probe_eager_poisoned']['rows']: print('  ', r['step'], round(r['loss'],4), r['n_bad_grads'], r['bad_grads'][:6], r['n_bad_weights'])
"
echo done
