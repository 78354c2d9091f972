#!/bin/bash
# Round-2 check 32: fused stem BN+ReLU+maxpool with a 2048-block gather reduction (numerics +
# per-kernel times under rocprofv3), BERT-base whole-step graph vs eager in the graph tests,
# then the N=1 bench with BERT jobs replaying step graphs.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c32
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_batchnorm_gpu.py tests/test_stepgraph_gpu.py -m gpu -x -q -k "maxpool or graph" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_stem -o stem -- python3 $R/benchmarks/bench_stem.py --only-bn-pool ) > $O/prof_stem.log 2>&1 || { tail -20 $O/prof_stem.log; exit 3; }
grep stem_bn $O/prof_stem.log
cp /tmp/prof_stem/stem_kernel_stats.csv $O/ 2>/dev/null || find /tmp/prof_stem -name "*kernel_stats.csv" -exec cp {} $O/stem_kernel_stats.csv \;
python3 -c "
import csv
rows=list(csv.DictReader(open('$O/stem_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:110])
"
timeout -k 10 600 python3 bench.py --out $O/bench_n1_detail.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 5; }
tail -1 $O/bench.log
