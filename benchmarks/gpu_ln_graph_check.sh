#!/bin/bash
# LayerNorm backward rewrite (numerics + BERT step) and the BERT whole-step hipGraph experiment.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "layer" --timeout 120 --timeout-method thread > gpurun_out/ln_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 > gpurun_out/bert_eager.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 --graph > gpurun_out/bert_graph.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/resnet_eager.log 2>&1 || exit $?
