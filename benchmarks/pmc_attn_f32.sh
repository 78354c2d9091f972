set -o pipefail
OUT=${PMC_OUT:-r4pa}
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_f32_target.py > $GRAFT_REPO_ROOT/gpurun_out/$OUT/pmc.log 2>&1
