#!/bin/bash
# Round-2 check 43: GELU fused into hipBLASLt GEMM epilogues (GELU_AUX_BIAS forward, DGELU
# backward) for the transformer FFN: numerics, graph replay, BERT-base A/B + kernel profile.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c43
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_ffn_gpu.py tests/test_layers_gpu.py tests/test_stepgraph_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 0 1; do
    VODA_GELU_EPILOGUE=$v timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 | sed "s/^{/{\"env\": \"VODA_GELU_EPILOGUE=$v\", /" >> $O/ab_epi.jsonl || exit 4
  done
done
cut -c1-140 $O/ab_epi.jsonl
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bert -o bert -- python3 $R/benchmarks/model_step.py --model bert-base --batch 64 --steps 10 --warmup 6 --profile-marker ) > $O/prof_bert.log 2>&1 || { tail -10 $O/prof_bert.log; exit 6; }
mkdir -p $O/prof_bert
python3 $R/benchmarks/trace_window_stats.py /tmp/prof_bert/bert_kernel_trace.csv $O/prof_bert/steady_kernel_stats.csv >> $O/prof_bert.log 2>&1 || exit 7
tail -1 $O/prof_bert.log
