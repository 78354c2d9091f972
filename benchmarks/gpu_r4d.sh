set -o pipefail
mkdir -p gpurun_out/r4d
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_f32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d/test_f32.log 2>&1 || { tail -40 gpurun_out/r4d/test_f32.log; exit 1; }
tail -2 gpurun_out/r4d/test_f32.log
timeout -k 10 300 python benchmarks/bench_resnet_fp32_convs.py --only-1x1 --out gpurun_out/r4d/convs1x1.jsonl > gpurun_out/r4d/convs.log 2>&1 || { tail -20 gpurun_out/r4d/convs.log; exit 1; }
tail -1 gpurun_out/r4d/convs.log
