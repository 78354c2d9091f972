set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 400 python -u -m pytest tests/test_attention_f32_gpu.py tests/test_xent_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/tests_f32attn.log 2>&1; rc=$?; tail -15 gpurun_out/r3c/tests_f32attn.log; [ $rc = 0 ] || exit $rc
bash benchmarks/gpu_lease.sh r3c step-bert-base-fp32 prof-bert-base-fp32
