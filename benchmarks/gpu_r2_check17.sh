#!/bin/bash
# Round-2 check 17: attention kernels staging up to 4 tiles per barrier pair (NT): numerics,
# BERT-base step A/B against the streaming kernels (VODA_ATTN_NT=1), per-kernel rocprof.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c17
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $R/gpurun_out/c17/pytest_attn.log 2>&1 || { tail -30 $R/gpurun_out/c17/pytest_attn.log; exit 2; }
tail -2 $R/gpurun_out/c17/pytest_attn.log
for rep in 1 2; do
  for env in "VODA_ATTN_NT=1" "VODA_ATTN_NT=4"; do
    env $env timeout -k 10 240 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 40 --warmup 6 | sed "s/^{/{\"env\": \"$env\", /" >> $R/gpurun_out/c17/ab_bert.jsonl || exit 4
  done
done
cat $R/gpurun_out/c17/ab_bert.jsonl
for nt in 1 4; do
  ( cd /tmp && VODA_ATTN_NT=$nt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_attn$nt -o attn$nt -- python3 $R/benchmarks/model_step.py --model bert-base --batch 64 --steps 10 --warmup 4 ) > $R/gpurun_out/c17/prof$nt.log 2>&1 || { tail -5 $R/gpurun_out/c17/prof$nt.log; exit 5; }
  f=$(find /tmp/prof_attn$nt -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/c17/attn_nt${nt}_kernel_stats.csv
  grep -i "attn_" $R/gpurun_out/c17/attn_nt${nt}_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
echo done
