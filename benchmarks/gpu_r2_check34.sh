#!/bin/bash
# Round-2 check 34: split-major wgrad block order (VODA_WGRAD_ORDER=1, default) vs the
# tile-major order: numerics of every wgrad path, per-shape times (BERT + ResNet-50 shapes),
# then BERT-base and ResNet-50 step A/B (alternating, same box).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c34
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_wgrad.py tests/test_conv1x1.py tests/test_conv3x3.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for v in 0 1; do
  VODA_WGRAD_ORDER=$v timeout -k 10 300 python3 -u benchmarks/bench_wgrad_fp32.py --no-blaslt > $O/micro_order$v.jsonl 2> $O/micro_order$v.err || { tail -5 $O/micro_order$v.err; exit 3; }
done
python3 -c "
import json
a=[json.loads(l) for l in open('$O/micro_order0.jsonl') if l.startswith('{')]
b=[json.loads(l) for l in open('$O/micro_order1.jsonl') if l.startswith('{')]
for x,y in zip(a,b): print(x['shape'], x['ours_us'], '->', y['ours_us'])
"
for rep in 1 2; do
  for v in 0 1; do
    VODA_WGRAD_ORDER=$v timeout -k 10 200 python3 -u benchmarks/model_step.py --model bert-base --steps 30 --warmup 5 | sed "s/^{/{\"env\": \"VODA_WGRAD_ORDER=$v\", /" >> $O/ab_order.jsonl || exit 4
    VODA_WGRAD_ORDER=$v timeout -k 10 300 python3 -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 | sed "s/^{/{\"env\": \"VODA_WGRAD_ORDER=$v\", /" >> $O/ab_order.jsonl || exit 5
  done
done
cat $O/ab_order.jsonl
