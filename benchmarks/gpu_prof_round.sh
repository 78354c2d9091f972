#!/bin/bash
# Counter pass on the wgrad stage loop, kernel-trace profile of the BERT step, and the N=1 bench.
set -o pipefail
mkdir -p gpurun_out/pmc gpurun_out/bert_prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --output-format csv -d gpurun_out/pmc/p1 -- python3 benchmarks/wgrad_one.py --splits 1 --variant 0 > gpurun_out/pmc/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --output-format csv -d gpurun_out/pmc/p2 -- python3 benchmarks/wgrad_one.py --splits 12 --variant 0 > gpurun_out/pmc/p2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bert_prof -- python3 benchmarks/model_step.py --model bert-base --steps 10 --warmup 5 --profile-marker > gpurun_out/bert_prof.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --out gpurun_out/bench_n1.json > gpurun_out/bench_n1.log 2>&1 || exit $?
