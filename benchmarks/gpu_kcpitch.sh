# Same-box A/B of the K-contiguous LDS pitch (96 B with swapped halves vs the padded 112 B): the
# two builds of _vodahip swap between model_step.py runs (one process each).
set -o pipefail
mkdir -p gpurun_out/kc
SO=vodascheduler_amd/_vodahip.cpython-310-x86_64-linux-gnu.so
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cp ab_so/ab_kc96.so $SO
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitgemm_gpu.py > gpurun_out/kc/tests.log 2>&1 || { tail -30 gpurun_out/kc/tests.log; exit 1; }
tail -1 gpurun_out/kc/tests.log
timeout -k 10 240 python -u benchmarks/probe_fwd_kmajor.py --out gpurun_out/kc/fwd_probe_kc96.jsonl > gpurun_out/kc/probe96.log 2>&1 || exit 1
for m in bert-base resnet50; do
  for i in 1 2; do
    for v in 112 96; do
      cp ab_so/ab_kc$v.so $SO
      timeout -k 10 300 python -u benchmarks/model_step.py --model $m --steps 30 --warmup 10 --precision fp32 > gpurun_out/kc/$m-$v-$i.log 2>&1 || { tail -20 gpurun_out/kc/$m-$v-$i.log; exit 1; }
      echo "{\"pitch\": $v, \"rep\": $i, \"run\": $(grep '^{' gpurun_out/kc/$m-$v-$i.log | tail -1)}" | tee -a gpurun_out/kc/ab_kc_pitch.jsonl | cut -c1-150
    done
  done
done
cp ab_so/ab_kc96.so $SO
