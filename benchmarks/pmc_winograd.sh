# One PMC pass over benchmarks/bench_winograd.py (batch 64 keeps it short): MFMA busy, waits,
# LDS bank conflicts of the Winograd kernel next to MIOpen's igemm.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${PMC_OUT:-pmcw}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_winograd.py --batch 64 > $OUT/pmc.log 2>&1
