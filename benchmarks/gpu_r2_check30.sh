#!/bin/bash
# Round-2 check 30 (session re-entry): full GPU suite + smoke + N=1 bench on the current tree,
# plus the ResNet-50 / BERT-base / NMT single-GPU step times.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c30
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
for m in resnet50 bert-base transformer; do
  timeout -k 10 300 python3 -u benchmarks/model_step.py --model $m --steps 20 --warmup 5 > $O/step_$m.log 2>&1 || { tail -20 $O/step_$m.log; exit 4; }
  tail -1 $O/step_$m.log
done
timeout -k 10 600 python3 bench.py --out $O/bench_n1_detail.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 5; }
tail -1 $O/bench.log
