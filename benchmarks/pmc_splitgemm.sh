# Two PMC passes (8 SQ counters each, separate runs) over one split-bf16 GEMM shape and its
# hipBLASLt fp32 twin (benchmarks/sgemm_one.py): MFMA busy, VALU / LDS activity, waits.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${PMC_OUT:-pmcs}
ARGS=${SG_ARGS:---shape 8192,2304,768 --op fwd --variants 1,4 --blas}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/sgemm_one.py $ARGS > $OUT/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/sgemm_one.py $ARGS > $OUT/p2.log 2>&1
