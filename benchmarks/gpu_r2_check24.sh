#!/bin/bash
# Round-2 check 24: torch.profiler op tables (which aten op launches each library / PyTorch
# kernel, with input shapes) for ResNet-50 and BERT-base steps.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c24
mkdir -p $O
timeout -k 10 300 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 5 --warmup 5 --torch-profile $O/ops_resnet50.txt > $O/r50.log 2>&1 || { tail -20 $O/r50.log; exit 2; }
tail -1 $O/r50.log
timeout -k 10 300 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 5 --warmup 5 --torch-profile $O/ops_bert.txt > $O/bert.log 2>&1 || { tail -20 $O/bert.log; exit 3; }
tail -1 $O/bert.log
echo done
