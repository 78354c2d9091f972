#!/bin/bash
# Round-2 check 16: NMT Transformer with separate Q / KV cross-attention projections.
# Eager step time, then the replay diag at bs 64; only if that is clean, the bs-512 NaN probe
# and the graph step time.  Stops at the first problem.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c16
for rep in 1 2; do
  for env in "VODA_WGRAD_VARIANT=2" "VODA_WGRAD_AUTO=1"; do
    env $env timeout -k 10 240 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 30 --warmup 6 | sed "s/^{/{\"env\": \"$env\", /" >> $R/gpurun_out/c16/ab_wgrad_choice.jsonl || exit 1
  done
done
cat $R/gpurun_out/c16/ab_wgrad_choice.jsonl
timeout -k 10 150 python3 benchmarks/model_step.py --model transformer --batch 512 --steps 30 --warmup 5 > $R/gpurun_out/c16/eager.json || exit 2
cat $R/gpurun_out/c16/eager.json
timeout -k 10 150 python3 benchmarks/graph_diag.py --model transformer --batch 64 > $R/gpurun_out/c16/diag_bs64.json 2> $R/gpurun_out/c16/diag_bs64.err || { tail -5 $R/gpurun_out/c16/diag_bs64.err; exit 3; }
python3 -c "
import json, sys; d=json.load(open('$R/gpurun_out/c16/diag_bs64.json')); u=d['update_check']
bad=[b['param'] for r in d['replays'] for b in r['bad']]
print('frozen', [r['n_bad'] for r in d['replays']], bad[:6])
print('update state_rel', u['state_rel_err_max'], [round(v,4) for v in u['losses_eager']], [round(v,4) for v in u['losses_graph']])
sys.exit(1 if bad or not u['state_rel_err_max'] < 1e-2 else 0)
" || { echo "diag not clean: stopping before the bs-512 replays"; exit 4; }
timeout -k 10 150 python3 benchmarks/graph_diag.py --model transformer --batch 512 --nan-probe 4 --graph-only > $R/gpurun_out/c16/probe_bs512.json 2> $R/gpurun_out/c16/probe.err || { tail -5 $R/gpurun_out/c16/probe.err; exit 5; }
python3 -c "
import json; d=json.load(open('$R/gpurun_out/c16/probe_bs512.json'))
print('probe', [(r['step'], round(r['loss'],4), r['n_bad_grads']) for r in d['probe_graph']['rows']])
"
timeout -k 10 150 python3 benchmarks/model_step.py --model transformer --batch 512 --steps 30 --warmup 5 --graph > $R/gpurun_out/c16/graph.json || exit 6
cat $R/gpurun_out/c16/graph.json
echo done
