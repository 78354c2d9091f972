#!/bin/bash
# Round-2 check 12: is the convnet hipGraph replay failure tied to MIOpen's timing-based
# solver choice (exhaustive find)?  Repeated graph NaN probes with find mode and with
# immediate mode, for ResNet-50, ResNet-50-CIFAR and VGG16.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c12
probe() {  # tag model batch extra
  timeout -k 10 200 python3 benchmarks/graph_diag.py --model $2 --batch $3 --nan-probe 5 --graph-only $4 > $R/gpurun_out/c12/$1.json 2> $R/gpurun_out/c12/$1.err || { tail -5 $R/gpurun_out/c12/$1.err; return 3; }
  python3 -c "
import json; d=json.load(open('$R/gpurun_out/c12/$1.json'))
rows=d['probe_graph']['rows']; bad=[r['step'] for r in rows if r['n_bad_grads']]
print('$1', 'first_bad', bad[0] if bad else None, [round(r['loss'],3) for r in rows], rows[bad[0]]['bad_grads'][:4] if bad else [])
"
}
for i in 1 2 3; do
  probe r50_find_$i resnet50 64 "" || exit 3
  probe r50_imm_$i resnet50 64 --no-benchmark || exit 3
done
for i in 1 2; do
  probe cifar_find_$i resnet50-cifar 128 "" || exit 3
  probe vgg_find_$i vgg16 128 "" || exit 3
done
echo done
