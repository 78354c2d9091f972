#!/bin/bash
# Round-2 check 4: hipGraph capture validation of the convnets (gradients + real updates vs
# eager), graph vs eager step time of the launch-bound ones, smoke().
set -o pipefail
mkdir -p gpurun_out
for spec in "resnet50 64" "inceptionv3 128" "vgg16 128" "resnet50-cifar 128"; do
  set -- $spec
  timeout -k 10 300 python3 benchmarks/graph_diag.py --model $1 --batch $2 > gpurun_out/r2c4_graph_diag_$1.json 2> gpurun_out/r2c4_graph_diag_$1.err || { echo "diag $1 failed"; tail -5 gpurun_out/r2c4_graph_diag_$1.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r2c4_graph_diag_$1.json')); u=d['update_check']; print('$1', [r['n_bad'] for r in d['replays']], 'state_rel', u['state_rel_err_max'], 'loss e', [round(x,4) for x in u['losses_eager']], 'g', [round(x,4) for x in u['losses_graph']])"
done
for m in inceptionv3 vgg16; do
  timeout -k 10 240 python3 benchmarks/model_step.py --model $m --steps 30 --warmup 5 >> gpurun_out/r2c4_graph_steps.jsonl || exit 3
  timeout -k 10 240 python3 benchmarks/model_step.py --model $m --steps 30 --warmup 5 --graph >> gpurun_out/r2c4_graph_steps.jsonl || exit 3
done
cat gpurun_out/r2c4_graph_steps.jsonl
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 4
