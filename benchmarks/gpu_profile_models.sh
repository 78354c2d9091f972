# Per-model single-GPU step times + steady-state rocprofv3 kernel stats (run from the repo root
# on a GPU box).  Only the summaries are kept (full traces exceed what gpurun copies back).
export TMPDIR=/tmp
R=$PWD
MODELS=${MODELS:-"bert-base:64 resnet50:256"}
if [ -z "$SKIP_TIMING" ]; then
for mb in $MODELS; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 python benchmarks/model_step.py --model $m --batch $b >> gpurun_out/steps.log 2>&1 || exit 1
done
fi
cd /tmp
for mb in $MODELS; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$m -o $m -- python3 $R/benchmarks/model_step.py --model $m --batch $b --steps 10 --warmup 6 --profile-marker > $R/gpurun_out/prof_$m.log 2>&1 || exit 2
  mkdir -p $R/gpurun_out/prof_$m
  python3 $R/benchmarks/trace_window_stats.py /tmp/prof_$m/${m}_kernel_trace.csv $R/gpurun_out/prof_$m/${m}_steady_kernel_stats.csv >> $R/gpurun_out/prof_$m.log 2>&1 || exit 3
  find /tmp/prof_$m -name '*stats.csv' -exec cp {} $R/gpurun_out/prof_$m/ \;
done
echo done
