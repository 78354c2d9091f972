#!/bin/bash
# Round-2 check 39: MIOpen solver families for the convolutions left on MIOpen (3x3 fwd /
# input gradient, Cin = 64 layers, stem).  The asm implicit-GEMM GTC NHWC solvers accumulate
# with atomics and need a SubTensorOpWithScalar1d zero pass per call (~27 per ResNet-50 step,
# ~19 us each, profiles/raw/r2_torch_ops_resnet50_c33.txt).  A/B with those solvers disabled
# so MIOpen's exhaustive find picks from the rest (CK grouped-conv kernels); each config gets
# its own find-db directory.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c39
mkdir -p $O
cfgs=("base" "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0"
      "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0"
      "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0")
for rep in 1 2; do
  for i in 0 1 2 3; do
    c=${cfgs[$i]}
    e=""; [ "$c" != "base" ] && e="$c"
    env VODA_MIOPEN_DIR=/tmp/miopen_cfg$i $e timeout -k 10 300 python3 -u benchmarks/model_step.py --model resnet50 --steps 20 --warmup 5 | sed "s/^{/{\"env\": \"$c\", /" >> $O/ab_miopen.jsonl || exit 4
  done
done
cat $O/ab_miopen.jsonl | cut -c1-260
