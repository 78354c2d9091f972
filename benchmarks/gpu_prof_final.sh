#!/bin/bash
# Steady-state rocprofv3 kernel stats of both flagship models with the current code.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out
run() {  # name, model, batch
  local name=$1 m=$2 b=$3
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o $name -- python3 $R/benchmarks/model_step.py --model $m --batch $b --steps 10 --warmup 6 --profile-marker ) > $R/gpurun_out/prof_$name.log 2>&1 || return 2
  mkdir -p $R/gpurun_out/prof_$name
  python3 $R/benchmarks/trace_window_stats.py /tmp/prof_$name/${name}_kernel_trace.csv $R/gpurun_out/prof_$name/steady_kernel_stats.csv >> $R/gpurun_out/prof_$name.log 2>&1 || return 3
}
run resnet50 resnet50 256 || exit $?
run bert bert-base 64 || exit $?
