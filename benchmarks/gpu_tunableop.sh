# Produce var/tunableop/fp32.csv (TunableOp: fastest hipBLASLt solution per fp32 GEMM shape of
# the bench workloads) and A/B it.  Results land in gpurun_out/r4n/ -- copy fp32.csv into
# var/tunableop/ to ship it.
set -o pipefail
OUT=gpurun_out/r4n
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for m in bert-base resnet50; do
  VODA_TUNABLEOP_TUNE=1 VODA_TUNABLEOP_DIR=$PWD/$OUT timeout -k 10 700 python -u benchmarks/model_step.py --model $m \
    --steps 5 --warmup 3 --precision fp32 > $OUT/tune_$m.log 2>&1 || { tail -20 $OUT/tune_$m.log; exit 1; }
  tail -1 $OUT/tune_$m.log
done
wc -l $OUT/fp32.csv
for m in bert-base resnet50; do
  VODA_TUNABLEOP=0 timeout -k 10 300 python -u benchmarks/model_step.py --model $m --steps 20 --warmup 5 \
    --precision fp32 > $OUT/off_$m.log 2>&1 || exit 1
  VODA_TUNABLEOP_DIR=$PWD/$OUT timeout -k 10 300 python -u benchmarks/model_step.py --model $m --steps 20 --warmup 5 \
    --precision fp32 > $OUT/on_$m.log 2>&1 || exit 1
  grep -h '^{' $OUT/off_$m.log $OUT/on_$m.log
done
