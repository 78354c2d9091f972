#!/bin/bash
# Round-2 check 37 = checks 35 + 36 in one call (strided GradSink A/B, wgrad re-sweep).
set -o pipefail
bash benchmarks/gpu_r2_check35.sh || exit $?
bash benchmarks/gpu_r2_check36.sh || exit $?
