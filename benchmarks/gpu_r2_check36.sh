#!/bin/bash
# Round-2 check 36: wgrad variant x split re-sweep under the split-major block order (the
# optimum may have moved now that an XCD's blocks share operand stages).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c36
mkdir -p $O
timeout -k 10 600 python3 -u benchmarks/bench_wgrad_fp32.py --sweep --variants 1,2,3 --split-mults 0.5,0.75,1,1.25,1.5,2 > $O/sweep.jsonl 2> $O/sweep.err || { tail -5 $O/sweep.err; exit 3; }
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l); print(d['shape'], 'default', d['ours_us'], 'best', d['best_us'], 'v', d['best_variant'], 's', d['best_splits'])
"
