#!/bin/bash
# Round-2 check 27: fused cross-entropy + padded BERT vocab + split-K head dgrad + flat-gradient
# embedding.  GPU tests of the new ops and of the transformer models, then eager step times
# of BERT-base and the NMT Transformer (new default vs VODA_FUSED_XENT=0 VODA_SPLIT_DGRAD=0,
# interleaved).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c27
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_xent_gpu.py tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
for rep in 1 2; do
  for env in "VODA_NONE=1" "VODA_FUSED_XENT=0 VODA_SPLIT_DGRAD=0 VODA_FUSED_EMBEDDING=0"; do
    env $env timeout -k 10 200 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 40 --warmup 6 | sed "s/^{/{\"env\": \"$env\", /" >> $O/ab.jsonl || exit 3
    env $env timeout -k 10 200 python3 benchmarks/model_step.py --model transformer --batch 512 --steps 40 --warmup 6 | sed "s/^{/{\"env\": \"$env\", /" >> $O/ab.jsonl || exit 4
  done
done
cat $O/ab.jsonl
echo done
