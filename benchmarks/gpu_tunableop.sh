# Produce var/tunableop/{fp32,bf16}.csv (TunableOp: fastest hipBLASLt solution per GEMM shape of
# the bench workloads) and A/B them.  Results land in gpurun_out/r4n/ -- copy the csv files
# into var/tunableop/ to ship them.
set -o pipefail
OUT=gpurun_out/r4n
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for prec in fp32 bf16-amp; do
  for m in bert-base resnet50; do
    VODA_TUNABLEOP_TUNE=1 VODA_TUNABLEOP_DIR=$PWD/$OUT timeout -k 10 700 python -u benchmarks/model_step.py --model $m \
      --steps 5 --warmup 3 --precision $prec > $OUT/tune_${m}_$prec.log 2>&1 || { tail -20 $OUT/tune_${m}_$prec.log; exit 1; }
    tail -1 $OUT/tune_${m}_$prec.log
  done
done
wc -l $OUT/*.csv
for prec in fp32 bf16-amp; do
  for m in bert-base resnet50; do
    VODA_TUNABLEOP=0 timeout -k 10 300 python -u benchmarks/model_step.py --model $m --steps 20 --warmup 5 \
      --precision $prec > $OUT/off_${m}_$prec.log 2>&1 || exit 1
    VODA_TUNABLEOP_DIR=$PWD/$OUT timeout -k 10 300 python -u benchmarks/model_step.py --model $m --steps 20 --warmup 5 \
      --precision $prec > $OUT/on_${m}_$prec.log 2>&1 || exit 1
    grep -h '^{' $OUT/off_${m}_$prec.log $OUT/on_${m}_$prec.log
  done
done
