#!/bin/bash
# Round-2 check 6: BN reduction passes on buffer-descriptor loads (8 waves/SIMD), grid cap and
# sweep-order A/B: numerics, per-kernel rocprof of the BN micro-benchmark per tuning, ResNet-50
# step A/B; ResNet-50 bs-256 graph trajectory vs an eager-vs-eager control.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c6
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batchnorm_gpu.py > $R/gpurun_out/c6/pytest_bn.log 2>&1 || { tail -30 $R/gpurun_out/c6/pytest_bn.log; exit 2; }
tail -2 $R/gpurun_out/c6/pytest_bn.log
for t in 1,1024,0 1,2048,0 1,2048,1 0,2048,0; do
  n=bn_${t//,/_}
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$n -o $n -- python3 $R/benchmarks/bench_bn_passes.py --tuning $t ) > $R/gpurun_out/c6/$n.log 2>&1 || { tail -20 $R/gpurun_out/c6/$n.log; exit 3; }
  cp /tmp/prof_$n/${n}_kernel_stats.csv $R/gpurun_out/c6/ 2>/dev/null || find /tmp/prof_$n -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/c6/${n}_kernel_stats.csv \;
done
for rep in 1 2; do
  for env in "VODA_BN_BLOCKS=1024" "VODA_BN_BLOCKS=2048" "VODA_BN_SWEEP=1"; do
    env $env timeout -k 10 240 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 20 --warmup 6 | sed "s/^{/{\"env\": \"$env\", /" >> $R/gpurun_out/c6/ab_resnet50.jsonl || exit 4
  done
done
cat $R/gpurun_out/c6/ab_resnet50.jsonl
timeout -k 10 400 python3 benchmarks/graph_diag.py --model resnet50 --batch 256 --update-steps 30 --skip-frozen --control > $R/gpurun_out/c6/graph_diag_resnet50_bs256.json 2> $R/gpurun_out/c6/graph_diag.err || { tail -5 $R/gpurun_out/c6/graph_diag.err; exit 5; }
python3 -c "
import json; d=json.load(open('$R/gpurun_out/c6/graph_diag_resnet50_bs256.json'))
for k in ('update_check','update_control'):
    u=d[k]; print(k, 'state_rel', u['state_rel_err_max']); print(' eager', [round(v,3) for v in u['losses_eager']]); print(' other', [round(v,3) for v in u['losses_graph']])
"
echo done
