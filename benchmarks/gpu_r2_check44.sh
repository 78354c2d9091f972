#!/bin/bash
# Round-2 check 44: hipBLASLt epilogue capability probe on gfx950 (bf16).
set -o pipefail
O=$PWD/gpurun_out/c44
mkdir -p $O
timeout -k 10 120 python3 -u benchmarks/blaslt_epilogue_probe.py > $O/probe.jsonl 2> $O/probe.err || { tail -5 $O/probe.err; exit 2; }
cat $O/probe.jsonl
