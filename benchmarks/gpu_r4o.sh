# fp32 GEMM numerics + 1x1 microbench, TunableOp production + A/B, smoke,
# fp32 attention waves-per-workgroup A/B
set -o pipefail
mkdir -p gpurun_out/r4o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv1x1_f32_gpu.py || exit 1
timeout -k 10 300 python benchmarks/bench_resnet_fp32_convs.py --only-1x1 --out gpurun_out/r4o/convs_1x1.jsonl > gpurun_out/r4o/convs_1x1.log 2>&1 || exit 1
bash benchmarks/gpu_tunableop.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash benchmarks/gpu_lease.sh r4o env:VODA_ATTN_F32_MAXW=2 prof-bert-base-fp32 env:VODA_ATTN_F32_MAXW=1 prof-bert-base-fp32 || exit 1
for f in gpurun_out/r4o/*.md; do echo "$f"; sed -n 3p "$f"; grep attn_f32 "$f" | cut -c1-120; done
