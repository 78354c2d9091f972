# Per-model single-GPU step times + rocprofv3 kernel stats (run from the repo root on a GPU box).
# Keeps only the *_stats.csv summaries (the full traces exceed what gpurun copies back).
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
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$m -o $m -- python3 $R/benchmarks/model_step.py --model $m --batch $b --steps 10 --warmup 3 > $R/gpurun_out/prof_$m.log 2>&1 || exit 2
  mkdir -p $R/gpurun_out/prof_$m
  find /tmp/prof_$m -name '*stats.csv' -exec cp {} $R/gpurun_out/prof_$m/ \;
  du -sh /tmp/prof_$m; find /tmp/prof_$m -type f | head -20
done
echo done
