#!/bin/bash
# Round-2 check 10: per-convolution hipGraph replay probe with MIOpen exhaustive find
# (cudnn.benchmark, as the convnet workloads run), plus the kernel names of the suspect case.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/c10
timeout -k 10 500 python3 benchmarks/graph_conv_probe.py --steps 6 --benchmark > $R/gpurun_out/c10/conv_probe_bench.jsonl 2> $R/gpurun_out/c10/conv_probe.err || { tail -5 $R/gpurun_out/c10/conv_probe.err; exit 3; }
python3 -c "
import json
for l in open('$R/gpurun_out/c10/conv_probe_bench.jsonl'):
    d=json.loads(l); print(d['case'], d['path'], 'first_bad', d['first_bad_step'], [(r['grad_finite'], '%.2g'%r['grad_rel'], '%.2g'%r['weight_rel']) for r in d['rows']])
"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c10 -o c10 -- python3 $R/benchmarks/graph_conv_probe.py --steps 2 --benchmark --only "l1.conv3" ) > $R/gpurun_out/c10/prof.log 2>&1 || { tail -20 $R/gpurun_out/c10/prof.log; exit 4; }
find /tmp/prof_c10 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/c10/l1conv3_kernel_stats.csv \;
cut -d, -f1-3 $R/gpurun_out/c10/l1conv3_kernel_stats.csv | cut -c1-200
echo done
