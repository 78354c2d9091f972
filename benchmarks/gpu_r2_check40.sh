#!/bin/bash
# Round-2 check 40 = checks 38 + 39 in one call (attention mask staging, MIOpen solver A/B).
set -o pipefail
bash benchmarks/gpu_r2_check38.sh || exit $?
bash benchmarks/gpu_r2_check39.sh || exit $?
