#!/bin/bash
# Round-2 check 35: stride-2 downsample input gradient handed through the GradSink as the
# subsampled tensor (conv1's GEMM writes beta = 0, then a strided add) instead of a zero-filled
# full-resolution scatter: numerics (bottleneck sink tests), ResNet-50 step A/B.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c35
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_conv1x1.py tests/test_layers_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 0 1; do
    VODA_STRIDED_SINK=$v timeout -k 10 300 python3 -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 | sed "s/^{/{\"env\": \"VODA_STRIDED_SINK=$v\", /" >> $O/ab_sink.jsonl || exit 4
  done
done
cat $O/ab_sink.jsonl
