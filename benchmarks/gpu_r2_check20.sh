#!/bin/bash
# Round-2 check 20: ResNet-50 step A/B of the BN reduction grid (1024 vs 256 blocks) and sweep
# order, interleaved.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c20
for rep in 1 2; do
  for env in "VODA_BN_BLOCKS=1024 VODA_BN_SWEEP=0" "VODA_BN_BLOCKS=256 VODA_BN_SWEEP=0" "VODA_BN_BLOCKS=256 VODA_BN_SWEEP=1"; do
    env $env timeout -k 10 240 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 30 --warmup 6 | sed "s/^{/{\"env\": \"$env\", /" >> $R/gpurun_out/c20/ab_bn_grid.jsonl || exit 4
  done
done
cat $R/gpurun_out/c20/ab_bn_grid.jsonl
echo done
