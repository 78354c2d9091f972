#!/usr/bin/env bash
# Which MIOpen solvers can run ResNet-50's fp32 3x3 forward convolutions on this GPU, and how
# fast: the find result in NHWC (the layout the models use) and NCHW, and the Winograd solvers
# forced one by one (MIOpen's Winograd kernels take NCHW only).  MIOpenDriver ships with ROCm.
#   gpurun -- bash benchmarks/miopen_solver_probe.sh TAG
set -o pipefail
TAG=${1:-miop}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen-probe-db
export MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen-probe-cache
D=/opt/rocm/bin/MIOpenDriver
# n c H W k: stage-1 (56x56x64) and stage-3 (14x14x256) 3x3 stride-1 layers at batch 256
for shape in "256 64 56 56 64" "256 256 14 14 256"; do
  read -r n c h w k <<< "$shape"
  base="conv -n $n -c $c -H $h -W $w -k $k -y 3 -x 3 -p 1 -q 1 -u 1 -v 1 -F 1 -t 1 -i 10 -V 0"
  for lay in NHWC NCHW; do
    name="$OUT/c${c}_h${h}_${lay}_find.log"
    echo "[probe] $shape $lay find"
    timeout -k 10 240 $D $base -I $lay -O $lay -f $lay > "$name" 2>&1 || { echo "rc=$? (see $name)"; }
    grep -E "GPU Kernel Time|Algorithm|Solution" "$name" | head -5
  done
  for sol in ConvBinWinogradRxSf2x3g1 ConvBinWinogradRxSf2x3 ConvBinWinogradRxSf3x2 ConvBinWinograd3x3U \
             ConvWinoFuryRxS_2_3 ConvMPBidirectWinograd_3_3 ConvAsmImplicitGemmGTCDynamicFwdXdlopsNHWC; do
    lay=NCHW
    [[ $sol == *NHWC ]] && lay=NHWC
    name="$OUT/c${c}_h${h}_${sol}.log"
    echo "[probe] $shape $sol"
    timeout -k 10 240 $D $base -I $lay -O $lay -f $lay -S $sol > "$name" 2>&1 || echo "rc=$?"
    grep -E "GPU Kernel Time|not applicable|Error|error" "$name" | head -3
  done
done
echo "[probe] done"
