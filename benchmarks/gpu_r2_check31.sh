#!/bin/bash
# Round-2 check 31: BN back-to-front reduction sweep (VODA_BN_SWEEP=2), row-per-block
# maxpool kernels and the fused stem BN+ReLU+maxpool (VODA_FUSED_BN_POOL) (numerics + ResNet-50 A/B), stem channel-padding micro-benchmark, then the
# BERT-base / NMT whole-step hipGraph replay checks with the flat-gradient embeddings.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c31
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_batchnorm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/bn_tests.log 2>&1 || { tail -30 $O/bn_tests.log; exit 2; }
tail -1 $O/bn_tests.log
timeout -k 10 200 python3 -u benchmarks/bench_stem.py > $O/stem.jsonl 2> $O/stem.err || { tail -10 $O/stem.err; exit 3; }
cat $O/stem.jsonl
for rep in 1 2; do
  for env in "VODA_BN_SWEEP=1 VODA_FUSED_BN_POOL=0" "VODA_BN_SWEEP=2 VODA_FUSED_BN_POOL=0" "VODA_BN_SWEEP=1 VODA_FUSED_BN_POOL=1" "VODA_BN_SWEEP=2 VODA_FUSED_BN_POOL=1"; do
    env $env timeout -k 10 300 python3 -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 | sed "s/^{/{\"env\": \"$env\", /" >> $O/ab_sweep.jsonl || exit 4
  done
done
cat $O/ab_sweep.jsonl
check() {  # diag json -> exit 1 unless frozen grads exact and real-update trajectory equal
python3 -c "
import json, sys; d=json.load(open('$1')); u=d['update_check']
bad=[b['param'] for r in d['replays'] for b in r['bad']]
print('$1', 'frozen', [r['n_bad'] for r in d['replays']], bad[:6], 'update state_rel', u['state_rel_err_max'])
print(' losses', [round(v,4) for v in u['losses_eager']], [round(v,4) for v in u['losses_graph']])
sys.exit(1 if bad or not u['state_rel_err_max'] < 1e-2 else 0)
"
}
timeout -k 10 200 python3 benchmarks/graph_diag.py --model bert-base --batch 64 > $O/diag_bert_bs64.json 2> $O/diag_bert.err || { grep -v "^frame" $O/diag_bert.err | tail -6; exit 5; }
check $O/diag_bert_bs64.json || exit 6
for rep in 1 2; do
  for g in "" "--graph"; do
    timeout -k 10 200 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 40 --warmup 6 $g >> $O/ab_graph.jsonl || exit 7
  done
done
cat $O/ab_graph.jsonl
timeout -k 10 200 python3 benchmarks/graph_diag.py --model transformer --batch 512 > $O/diag_nmt_bs512.json 2> $O/diag_nmt.err || { grep -v "^frame" $O/diag_nmt.err | tail -6; exit 8; }
check $O/diag_nmt_bs512.json || exit 9
for rep in 1 2; do
  for g in "" "--graph"; do
    timeout -k 10 200 python3 benchmarks/model_step.py --model transformer --batch 512 --steps 40 --warmup 6 $g >> $O/ab_graph.jsonl || exit 10
  done
done
tail -4 $O/ab_graph.jsonl
echo done
