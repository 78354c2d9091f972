#!/bin/bash
# Steady-state kernel profile of the ResNet-50 step with the implicit-GEMM 3x3 weight gradient
# on and off: per-kernel stats + per-dispatch rows of the weight-gradient kernels.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out
run() {  # name, env assignment
  local name=$1 envset=$2
  ( export $envset; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o $name -- python3 $R/benchmarks/model_step.py --model resnet50 --batch 256 --steps 4 --warmup 6 --profile-marker ) > $R/gpurun_out/prof_$name.log 2>&1 || return 2
  mkdir -p $R/gpurun_out/prof_$name
  python3 $R/benchmarks/trace_window_stats.py /tmp/prof_$name/${name}_kernel_trace.csv $R/gpurun_out/prof_$name/steady_kernel_stats.csv >> $R/gpurun_out/prof_$name.log 2>&1 || return 3
  python3 $R/benchmarks/trace_dispatches.py /tmp/prof_$name/${name}_kernel_trace.csv $R/gpurun_out/prof_$name/wgrad_dispatches.csv wgrad igemm_wrw SubTensorOp >> $R/gpurun_out/prof_$name.log 2>&1 || return 4
}
run c3on VODA_CONV_WGRAD=1 || exit $?
[ -n "$ONLY_ON" ] || run c3off VODA_CONV_WGRAD=0 || exit $?
