#!/bin/bash
# Round-2 check 13: full GPU test suite + smoke after the BN / dropout / hybrid-1x1 changes;
# ResNet-50 A/B of the hybrid Cin<128 1x1 weight-gradient path.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c13
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/c13/pytest_gpu.log 2>&1 || { tail -40 $R/gpurun_out/c13/pytest_gpu.log; exit 2; }
tail -3 $R/gpurun_out/c13/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/gpurun_out/c13/smoke.log 2>&1 || { tail -20 $R/gpurun_out/c13/smoke.log; exit 3; }
tail -1 $R/gpurun_out/c13/smoke.log
for rep in 1 2; do
  for env in "VODA_CONV1X1_HYBRID=0" "VODA_CONV1X1_HYBRID=1"; do
    env $env timeout -k 10 240 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 30 --warmup 6 | sed "s/^{/{\"env\": \"$env\", /" >> $R/gpurun_out/c13/ab_hybrid.jsonl || exit 4
  done
done
cat $R/gpurun_out/c13/ab_hybrid.jsonl
echo done
