#!/bin/bash
# Round-2 check 25: BERT-base under whole-step hipGraph replay (never evaluated before).
# Replay diag at bs 16 (frozen gradients + real-update trajectory vs eager + eager control);
# only if clean, the NaN probe at the job batch (bs 64), then graph vs eager step time
# (interleaved).  Stops at the first problem.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c25
mkdir -p $O
timeout -k 10 200 python3 benchmarks/graph_diag.py --model bert-base --batch 16 --control > $O/diag_bs16.json 2> $O/diag_bs16.err || { tail -5 $O/diag_bs16.err; exit 3; }
python3 -c "
import json, sys; d=json.load(open('$O/diag_bs16.json')); u=d['update_check']
bad=[b['param'] for r in d['replays'] for b in r['bad']]
print('frozen', [r['n_bad'] for r in d['replays']], bad[:6])
print('update state_rel', u['state_rel_err_max'], [round(v,4) for v in u['losses_eager']], [round(v,4) for v in u['losses_graph']])
sys.exit(1 if bad or not u['state_rel_err_max'] < 1e-2 else 0)
" || { echo "diag not clean: stopping before the bs-64 replays"; exit 4; }
timeout -k 10 200 python3 benchmarks/graph_diag.py --model bert-base --batch 64 --nan-probe 6 --graph-only > $O/probe_bs64.json 2> $O/probe.err || { tail -5 $O/probe.err; exit 5; }
python3 -c "
import json; d=json.load(open('$O/probe_bs64.json'))
print('probe', [(r['step'], round(r['loss'],4), r['n_bad_grads']) for r in d['probe_graph']['rows']])
"
for rep in 1 2; do
  timeout -k 10 200 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 40 --warmup 6 >> $O/ab_graph.jsonl || exit 6
  timeout -k 10 200 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 40 --warmup 6 --graph >> $O/ab_graph.jsonl || exit 7
done
cat $O/ab_graph.jsonl
echo done
