#!/bin/bash
# Round-2 check 14: NMT Transformer under whole-step hipGraph (fused attention path since
# round 2): frozen-gradient replay diag + real-update check (bs 64), NaN probe at the job
# batch (bs 512), then eager vs graph step time.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c14
timeout -k 10 150 python3 benchmarks/graph_diag.py --model transformer --batch 64 > $R/gpurun_out/c14/diag_bs64.json 2> $R/gpurun_out/c14/diag_bs64.err || { tail -5 $R/gpurun_out/c14/diag_bs64.err; exit 2; }
python3 -c "
import json; d=json.load(open('$R/gpurun_out/c14/diag_bs64.json')); u=d['update_check']
print('frozen', [r['n_bad'] for r in d['replays']], [b['param'] for r in d['replays'] for b in r['bad']][:6])
print('update state_rel', u['state_rel_err_max'], [round(v,4) for v in u['losses_eager']], [round(v,4) for v in u['losses_graph']])
"
timeout -k 10 150 python3 benchmarks/graph_diag.py --model transformer --batch 512 --nan-probe 6 --graph-only > $R/gpurun_out/c14/probe_bs512.json 2> $R/gpurun_out/c14/probe.err || { tail -5 $R/gpurun_out/c14/probe.err; exit 3; }
python3 -c "
import json; d=json.load(open('$R/gpurun_out/c14/probe_bs512.json'))
print('probe', [(r['step'], round(r['loss'],4), r['n_bad_grads']) for r in d['probe_graph']['rows']])
"
for g in "" "--graph"; do
  timeout -k 10 150 python3 benchmarks/model_step.py --model transformer --batch 512 --steps 30 --warmup 5 $g >> $R/gpurun_out/c14/steps.jsonl || exit 4
done
cat $R/gpurun_out/c14/steps.jsonl
echo done
