# split-K reduce with slab groups: numerics, then ResNet-50 / BERT-base fp32 step A/B (automatic vs one group)
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/red_tests.log 2>&1 && \
bash benchmarks/gpu_lease.sh r6d abset:vodascheduler_amd.ops.splitgemm:REDUCE_GROUPS_AUTO:resnet50-fp32:2 abset:vodascheduler_amd.ops.splitgemm:REDUCE_GROUPS_AUTO:bert-base-fp32:2
