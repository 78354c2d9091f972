#!/bin/bash
# Round-2 check 5: VGG16 with the separate conv-bias op under hipGraph (diag), graph vs eager
# step times + capture cost for the ResNets / VGG16.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 benchmarks/graph_diag.py --model vgg16 --batch 128 > gpurun_out/r2c5_graph_diag_vgg16.json 2> gpurun_out/r2c5_graph_diag_vgg16.err || { tail -5 gpurun_out/r2c5_graph_diag_vgg16.err; exit 2; }
python3 -c "import json; d=json.load(open('gpurun_out/r2c5_graph_diag_vgg16.json')); u=d['update_check']; print('vgg16', [r['n_bad'] for r in d['replays']], [b['param'] for r in d['replays'] for b in r['bad']][:10], 'state_rel', u['state_rel_err_max'], u['losses_eager'], u['losses_graph'])"
for spec in "resnet50 256" "resnet50-cifar 128" "vgg16 128" "resnet18 256"; do
  set -- $spec
  for g in "" "--graph"; do
    timeout -k 10 240 python3 benchmarks/model_step.py --model $1 --batch $2 --steps 30 --warmup 5 $g >> gpurun_out/r2c5_graph_steps.jsonl || exit 3
  done
done
cat gpurun_out/r2c5_graph_steps.jsonl
