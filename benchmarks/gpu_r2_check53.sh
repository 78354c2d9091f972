#!/bin/bash
# Round-2 check 53 (final validation of the session tree: + large-head-dim attention direct loads, fold cast): full GPU suite + smoke,
# BERT-base eager vs graph, N=1 bench with detail, steady-state rocprofv3 kernel stats of
# ResNet-50 / BERT-base.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c53
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
for g in "" "--graph" "" "--graph"; do
  timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --batch 64 --steps 40 --warmup 6 $g >> $O/bert_graph_ab.jsonl || exit 4
done
cut -c1-120 $O/bert_graph_ab.jsonl
timeout -k 10 600 python3 bench.py --out $O/bench_n1_detail.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 5; }
tail -1 $O/bench.log
run() {  # name, model, batch
  local name=$1 m=$2 b=$3
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o $name -- python3 $R/benchmarks/model_step.py --model $m --batch $b --steps 10 --warmup 6 --profile-marker ) > $O/prof_$name.log 2>&1 || return 6
  mkdir -p $O/prof_$name
  python3 $R/benchmarks/trace_window_stats.py /tmp/prof_$name/${name}_kernel_trace.csv $O/prof_$name/steady_kernel_stats.csv >> $O/prof_$name.log 2>&1 || return 7
  tail -1 $O/prof_$name.log
}
run r2_resnet50_s6 resnet50 256 || exit $?
run r2_bert_s6 bert-base 64 || exit $?
echo done
