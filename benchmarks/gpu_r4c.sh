set -o pipefail
mkdir -p gpurun_out/r4c
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_f32_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4c/test_f32.log 2>&1 || { tail -40 gpurun_out/r4c/test_f32.log; exit 1; }
tail -3 gpurun_out/r4c/test_f32.log
timeout -k 10 300 python benchmarks/bench_resnet_fp32_convs.py --only-1x1 --out gpurun_out/r4c/convs1x1.jsonl > gpurun_out/r4c/convs.log 2>&1 || { tail -20 gpurun_out/r4c/convs.log; exit 1; }
timeout -k 10 300 python benchmarks/model_step.py --model resnet50 --precision fp32 --steps 20 --warmup 5 > gpurun_out/r4c/step_on.json 2> gpurun_out/r4c/step_on.err || { tail -20 gpurun_out/r4c/step_on.err; exit 1; }
VODA_CONV1X1_F32=0 timeout -k 10 300 python benchmarks/model_step.py --model resnet50 --precision fp32 --steps 20 --warmup 5 > gpurun_out/r4c/step_off.json 2> gpurun_out/r4c/step_off.err || { tail -20 gpurun_out/r4c/step_off.err; exit 1; }
cat gpurun_out/r4c/step_on.json gpurun_out/r4c/step_off.json
