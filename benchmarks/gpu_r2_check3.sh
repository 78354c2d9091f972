#!/bin/bash
# Round-2 check 3: streamed-tile attention tests (D=256, T<=512), NMT step fused vs
# materialised attention, hipGraph diagnostic of ResNet-50.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r2c3_pytest_attn.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r2c3_pytest_attn.log
tail -12 gpurun_out/r2c3_pytest_attn.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 python3 benchmarks/model_step.py --model transformer --batch 512 --steps 20 --warmup 5 > gpurun_out/r2c3_nmt_fused.json || exit 2
VODA_FLASH_MAX_D=128 timeout -k 10 240 python3 benchmarks/model_step.py --model transformer --batch 512 --steps 20 --warmup 5 > gpurun_out/r2c3_nmt_materialized.json || exit 2
cat gpurun_out/r2c3_nmt_fused.json gpurun_out/r2c3_nmt_materialized.json
timeout -k 10 300 python3 benchmarks/graph_diag.py --model resnet50 --batch 32 > gpurun_out/r2c3_graph_diag_resnet50.json 2> gpurun_out/r2c3_graph_diag.err
echo "graph diag rc=$?"
head -60 gpurun_out/r2c3_graph_diag_resnet50.json
# BN reduction-pass depth A/B (VODA_BN_UNROLL=0: round-1 depths)
for u in 0 1 0 1; do
  VODA_BN_UNROLL=$u timeout -k 10 300 python3 benchmarks/bench_bn_passes.py > gpurun_out/r2c3_bn_u$u.json || exit 3
  VODA_BN_UNROLL=$u timeout -k 10 240 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 20 --warmup 6 >> gpurun_out/r2c3_resnet_bn_ab.jsonl || exit 3
  echo "{\"bn_unroll\": $u}" >> gpurun_out/r2c3_resnet_bn_ab.jsonl
done
cat gpurun_out/r2c3_resnet_bn_ab.jsonl
python3 -c "import json;[print(u, json.load(open(f'gpurun_out/r2c3_bn_u{u}.json'))['per_step_fwd_ms'], json.load(open(f'gpurun_out/r2c3_bn_u{u}.json'))['per_step_bwd_ms']) for u in (0,1)]"
