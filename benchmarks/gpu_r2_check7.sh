#!/bin/bash
# Round-2 check 7: BN reduction loads A/B (buffer descriptors vs round-1 flat addresses) on the
# ResNet-50 step; per-step NaN probe of ResNet-50 graph replays (bs 256 and bs 64).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c7
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batchnorm_gpu.py > $R/gpurun_out/c7/pytest_bn.log 2>&1 || { tail -30 $R/gpurun_out/c7/pytest_bn.log; exit 2; }
tail -2 $R/gpurun_out/c7/pytest_bn.log
for rep in 1 2 3; do
  for env in "VODA_BN_LOADS=flat" "VODA_BN_LOADS=buffer"; do
    env $env timeout -k 10 240 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 30 --warmup 6 | sed "s/^{/{\"env\": \"$env\", /" >> $R/gpurun_out/c7/ab_resnet50.jsonl || exit 4
  done
done
cat $R/gpurun_out/c7/ab_resnet50.jsonl
for b in 256 64; do
  timeout -k 10 400 python3 benchmarks/graph_diag.py --model resnet50 --batch $b --nan-probe 12 > $R/gpurun_out/c7/nan_probe_resnet50_bs$b.json 2> $R/gpurun_out/c7/nan_probe_$b.err || { tail -5 $R/gpurun_out/c7/nan_probe_$b.err; exit 5; }
  python3 -c "
import json; d=json.load(open('$R/gpurun_out/c7/nan_probe_resnet50_bs$b.json'))
for k in ('probe_graph','probe_eager'):
    print(k, $b)
    for r in d[k]['rows']: print('  ', r['step'], round(r['loss'],4), r['n_bad_grads'], r['bad_grads'][:3], r['n_bad_weights'], r['bad_weights'][:3], r['top_grad_norms'])
"
done
echo done
