#!/bin/bash
# GPU check of the HIP tanh-GELU: numerics, BERT-base step with and without it
# (VODA_HIP_GELU, alternating, same box), then a steady-state kernel profile of BERT-base.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gelu_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  VODA_HIP_GELU=$v timeout -k 10 300 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 >> gpurun_out/bert_gelu_v$v.log 2>&1 || exit $?
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bert -o bert -- python3 $R/benchmarks/model_step.py --model bert-base --batch 64 --steps 10 --warmup 6 --profile-marker ) > $R/gpurun_out/prof_bert_gelu.log 2>&1 || exit 2
mkdir -p $R/gpurun_out/prof_bert_gelu
python3 $R/benchmarks/trace_window_stats.py /tmp/prof_bert/bert_kernel_trace.csv $R/gpurun_out/prof_bert_gelu/steady_kernel_stats.csv >> $R/gpurun_out/prof_bert_gelu.log 2>&1 || exit 3
