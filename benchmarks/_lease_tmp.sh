set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_attention_f32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e/tests_attn.log 2>&1; rc=$?; tail -3 gpurun_out/r3e/tests_attn.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for r in 1 0; do
    VODA_ATTN_RESIDENT=$r timeout -k 10 120 python -u benchmarks/bench_attention.py --fwd-only --iters 50 >> gpurun_out/r3e/attn_ab.jsonl || exit 5
    VODA_ATTN_RESIDENT=$r timeout -k 10 120 python -u benchmarks/bench_attention.py --iters 50 >> gpurun_out/r3e/attn_ab.jsonl || exit 6
  done
done
cat gpurun_out/r3e/attn_ab.jsonl
for r in 1 0; do
  VODA_ATTN_RESIDENT=$r timeout -k 10 200 python -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 2>/dev/null | sed "s/^{/{\"resident\": $r, /" >> gpurun_out/r3e/bert_ab.jsonl || exit 7
done
cat gpurun_out/r3e/bert_ab.jsonl
