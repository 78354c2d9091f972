#!/bin/bash
# fp32 vs bf16 flat gradients: step-time A/B (interleaved) + steady-state rocprofv3 kernel stats
# of ResNet-50 / BERT-base with the fp32 default; plus the node's GPU link topology (sysfs KFD
# topology, rocm-smi) for the placement topology model.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/topo
# --- topology probe (no GPU work)
( for f in /sys/class/kfd/kfd/topology/nodes/*/properties; do echo "== $f"; cat $f; done;
  for f in /sys/class/kfd/kfd/topology/nodes/*/io_links/*/properties; do echo "== $f"; cat $f; done ) \
  > $R/gpurun_out/topo/kfd_topology.txt 2>&1
timeout 60 rocm-smi --showtopo > $R/gpurun_out/topo/rocm_smi_showtopo.txt 2>&1
timeout 60 amd-smi topology > $R/gpurun_out/topo/amd_smi_topology.txt 2>&1
ls /sys/class/drm > $R/gpurun_out/topo/drm.txt 2>&1
for d in /sys/class/drm/card*/device; do echo "$d $(cat $d/numa_node 2>/dev/null) $(cat $d/local_cpulist 2>/dev/null)"; done >> $R/gpurun_out/topo/drm.txt 2>&1
# --- A/B step time
for rep in 1 2; do
  for g in fp32 bf16; do
    timeout -k 10 240 python3 benchmarks/model_step.py --model resnet50 --batch 256 --steps 20 --warmup 6 --grad-dtype $g >> $R/gpurun_out/ab_gradprec.jsonl || exit 2
    timeout -k 10 240 python3 benchmarks/model_step.py --model bert-base --batch 64 --steps 30 --warmup 6 --grad-dtype $g >> $R/gpurun_out/ab_gradprec.jsonl || exit 2
  done
done
cat $R/gpurun_out/ab_gradprec.jsonl
# --- profiles (fp32 default)
run() {  # name, model, batch
  local name=$1 m=$2 b=$3
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o $name -- python3 $R/benchmarks/model_step.py --model $m --batch $b --steps 10 --warmup 6 --profile-marker ) > $R/gpurun_out/prof_$name.log 2>&1 || return 2
  mkdir -p $R/gpurun_out/prof_$name
  python3 $R/benchmarks/trace_window_stats.py /tmp/prof_$name/${name}_kernel_trace.csv $R/gpurun_out/prof_$name/steady_kernel_stats.csv >> $R/gpurun_out/prof_$name.log 2>&1 || return 3
}
run r2_resnet50_fp32g resnet50 256 || exit $?
run r2_bert_fp32g bert-base 64 || exit $?
echo done
