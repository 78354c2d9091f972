#!/bin/bash
# Round-2 check 18: rotated transposed LDS images in the attention kernels: numerics, isolated
# fwd+bwd time, bank-conflict counters, BERT-base and NMT step times.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c18
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $R/gpurun_out/c18/pytest_attn.log 2>&1 || { tail -30 $R/gpurun_out/c18/pytest_attn.log; exit 2; }
tail -2 $R/gpurun_out/c18/pytest_attn.log
timeout -k 10 120 python3 benchmarks/bench_attention.py --iters 20 | tee $R/gpurun_out/c18/time.json || exit 3
( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc_lds -o lds -- python3 $R/benchmarks/bench_attention.py --iters 3 ) > $R/gpurun_out/c18/pmc.log 2>&1 || { tail -5 $R/gpurun_out/c18/pmc.log; exit 4; }
f=$(find /tmp/pmc_lds -name "*counter_collection.csv" | head -1); cp $f $R/gpurun_out/c18/lds.csv
python3 benchmarks/pmc_summary.py $R/gpurun_out/c18/lds.csv --match attn_
for m in "bert-base 64" "transformer 512"; do
  set -- $m
  timeout -k 10 240 python3 benchmarks/model_step.py --model $1 --batch $2 --steps 40 --warmup 6 >> $R/gpurun_out/c18/steps.jsonl || exit 5
done
cat $R/gpurun_out/c18/steps.jsonl
echo done
