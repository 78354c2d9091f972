#!/bin/bash
# Round-2 check 21: PyTorch TunableOp (hipBLASLt/rocBLAS solution search per GEMM shape) on the
# ResNet-50 and BERT-base steps: tune once, then time with the tuned table vs without.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c21
for m in "resnet50 256" "bert-base 64"; do
  set -- $m
  timeout -k 10 240 python3 benchmarks/model_step.py --model $1 --batch $2 --steps 30 --warmup 6 | sed 's/^{/{"tunableop": "off", /' >> $R/gpurun_out/c21/steps.jsonl || exit 2
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$R/gpurun_out/c21/tunableop_$1.csv \
    timeout -k 10 600 python3 benchmarks/model_step.py --model $1 --batch $2 --steps 5 --warmup 3 > $R/gpurun_out/c21/tune_$1.log 2>&1 || { tail -5 $R/gpurun_out/c21/tune_$1.log; exit 3; }
  ls $R/gpurun_out/c21/
  f=$(ls $R/gpurun_out/c21/tunableop_$1*.csv | head -1)
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$f \
    timeout -k 10 240 python3 benchmarks/model_step.py --model $1 --batch $2 --steps 30 --warmup 6 | sed 's/^{/{"tunableop": "tuned", /' >> $R/gpurun_out/c21/steps.jsonl || exit 4
  timeout -k 10 240 python3 benchmarks/model_step.py --model $1 --batch $2 --steps 30 --warmup 6 | sed 's/^{/{"tunableop": "off", /' >> $R/gpurun_out/c21/steps.jsonl || exit 2
done
cat $R/gpurun_out/c21/steps.jsonl
echo done
