set -o pipefail
timeout -k 10 300 python benchmarks/model_step.py --model resnet50 --batch 256 --cudnn-benchmark --warmup 8 2>&1 | grep model
mkdir -p gpurun_out/tunableop
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop/tunableop_results%d.csv
timeout -k 10 500 python benchmarks/model_step.py --model bert-base --batch 64 --warmup 5 2>&1 | grep model
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 300 python benchmarks/model_step.py --model bert-base --batch 64 --warmup 5 2>&1 | grep model
ls -la gpurun_out/tunableop
