#!/bin/bash
# Round-2 PMC passes (rocprofv3 --pmc, one counter group per run, kernel names only):
# BatchNorm passes on the largest ResNet-50 shapes, and the split-K wgrad kernel on the
# BERT-base shapes.  Counter limits per pass: <= 8 SQ, <= 4 TCC, <= 2 GRBM.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/pmc
pass() {  # tag, program args..., counters in $PMC
  local tag=$1; shift
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d /tmp/pmc_$tag -o $tag -- "$@" ) > $R/gpurun_out/pmc/$tag.log 2>&1 || { tail -5 $R/gpurun_out/pmc/$tag.log; return 3; }
  f=$(find /tmp/pmc_$tag -name "*counter_collection.csv" | head -1)
  cp $f $R/gpurun_out/pmc/$tag.csv
  python3 $R/benchmarks/pmc_summary.py $R/gpurun_out/pmc/$tag.csv --match "$MATCH" > $R/gpurun_out/pmc/$tag.md
}
BN="python3 $R/benchmarks/bench_bn_passes.py --shapes 1,2,10 --iters 3"
WG="python3 $R/benchmarks/bench_wgrad_fp32.py --only bert --no-blaslt"
MATCH=bn_ PMC="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE" pass bn_traffic $BN || exit 3
MATCH=bn_ PMC="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" pass bn_stalls $BN || exit 3
MATCH=wgrad PMC="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" pass wgrad_mfma $WG || exit 3
MATCH=wgrad PMC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" pass wgrad_traffic $WG || exit 3
cat $R/gpurun_out/pmc/*.md
echo done
