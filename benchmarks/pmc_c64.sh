set -o pipefail
mkdir -p gpurun_out/${PMC_OUT:-r4y}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/${PMC_OUT:-r4y}/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_c64_wgrad.py > $GRAFT_REPO_ROOT/gpurun_out/${PMC_OUT:-r4y}/pmc.log 2>&1
