#!/bin/bash
# PMC passes of the fused attention kernels on the BERT-base shape (one counter group per run).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/pmc_attn
timeout -k 10 120 python3 benchmarks/bench_attention.py --iters 20 > $R/gpurun_out/pmc_attn/time.json || exit 2
cat $R/gpurun_out/pmc_attn/time.json
pass() {
  local tag=$1; shift
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d /tmp/pmc_$tag -o $tag -- "$@" ) > $R/gpurun_out/pmc_attn/$tag.log 2>&1 || { tail -5 $R/gpurun_out/pmc_attn/$tag.log; return 3; }
  f=$(find /tmp/pmc_$tag -name "*counter_collection.csv" | head -1)
  cp $f $R/gpurun_out/pmc_attn/$tag.csv
  python3 $R/benchmarks/pmc_summary.py $R/gpurun_out/pmc_attn/$tag.csv --match attn_ > $R/gpurun_out/pmc_attn/$tag.md
}
A="python3 $R/benchmarks/bench_attention.py --iters 3"
PMC="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" pass lds $A || exit 3
PMC="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE" pass valu $A || exit 3
PMC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" pass l2 $A || exit 3
cat $R/gpurun_out/pmc_attn/*.md
echo done
