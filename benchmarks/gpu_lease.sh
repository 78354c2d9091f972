#!/usr/bin/env bash
# One GPU lease, several named steps, each under its own time limit; the first failing step
# ends the lease (no retries: a fault, abort or timeout means read the logs, then fix).
#
#   gpurun --timeout 1200 -- bash benchmarks/gpu_lease.sh TAG STEP [STEP ...]
#
# Steps (outputs under gpurun_out/TAG/):
#   tests            pytest -m gpu (one process, per-test 120 s timeout)
#   smoke            __graft_entry__.smoke()
#   bench            bench.py N=1, driver flags (--steps 20 --warmup 5), with the FIFO control
#   bench-fp32       bench.py N=1 at the reference's precision (fp32)
#   step-MODEL[-fp32]        benchmarks/model_step.py timing of one model (resnet50, bert-base, ...)
#   prof-MODEL[-fp32]        rocprofv3 --kernel-trace --stats of 10 steps of one model
#   pmc-MODEL:COUNTERS       one rocprofv3 --pmc pass (comma-separated counters)
#   profset:MODULE:ATTR=VALUE:MODEL[-fp32]  prof-MODEL with one module switch set (model_step.py --set)
#   py:SCRIPT[:ARGS]         python benchmarks/SCRIPT ARGS (comma-separated args)
#   pytest:FILE[,ARGS]       pytest -m gpu of one test file (comma-separated extra args)
#   env:NAME=VALUE           export for the following steps (their logs get a "+NAME=VALUE" suffix)
#   ab:NAME:MODEL[-fp32]:REPS  interleaved same-box A/B of one env switch: model_step.py with
#                            NAME=1 then NAME=0, REPS times (30 timed steps each); one JSON line
#                            per run in ab-NAME-MODEL.jsonl
#   abset:MODULE:ATTR:MODEL[-fp32]:REPS  the same for a module-level switch (docs/kernels.md):
#                            model_step.py --set MODULE:ATTR=True, then =False
set -o pipefail
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
SUFFIX=""
mkdir -p "$OUT"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MIOPEN_USER_DB_PATH=${MIOPEN_USER_DB_PATH:-$PWD/var/miopen/db}
export MIOPEN_CUSTOM_CACHE_DIR=${MIOPEN_CUSTOM_CACHE_DIR:-/tmp/miopen-cache}

run() {  # run SECONDS NAME CMD...
  local secs=$1 name=$2
  shift 2
  name=$name$SUFFIX
  echo "[lease $(date +%T)] $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[lease $(date +%T)] $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  return $rc
}

for step in "$@"; do
  case "$step" in
    tests)
      run 600 tests python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $? ;;
    smoke)
      run 300 smoke python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      run 590 bench python -u bench.py --steps 20 --warmup 5 --out "$OUT/bench.json" || exit $? ;;
    bench-fp32)
      run 590 bench-fp32 python -u bench.py --steps 20 --warmup 5 --precision fp32 --out "$OUT/bench_fp32.json" \
        || exit $? ;;
    step-*)
      m=${step#step-}
      prec=bf16-amp
      if [[ $m == *-fp32 ]]; then m=${m%-fp32}; prec=fp32; fi
      # fp32 convolutions meet MIOpen's exhaustive find for the first time (minutes, silent):
      # MIOpen's own info log is the progress signal until the find-db holds the shapes
      if [[ $prec == fp32 ]]; then export MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5; fi
      run 900 "$step" python -u benchmarks/model_step.py --model "$m" --steps 20 --warmup 5 --precision "$prec"
      rc=$?
      unset MIOPEN_ENABLE_LOGGING MIOPEN_LOG_LEVEL
      [[ $rc == 0 ]] || exit $rc
      grep '^{' "$OUT/$step$SUFFIX.log" || true ;;
    miopen-save)  # the find-db / perf-db this lease added, to commit under var/miopen/db
      mkdir -p "$OUT/miopen_db" && cp "$MIOPEN_USER_DB_PATH"/*.txt "$OUT/miopen_db/" && ls -la "$OUT/miopen_db" ;;
    prof-*)
      m=${step#prof-}
      prec=bf16-amp
      if [[ $m == *-fp32 ]]; then m=${m%-fp32}; prec=fp32; fi
      R=$PWD
      st="$step$SUFFIX"  # env-suffixed outputs stay apart (A/B profiles in one lease)
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/$st" -o k -- \
          python3 "$R/benchmarks/model_step.py" --model "$m" --steps 10 --warmup 6 --precision "$prec" \
          --profile-marker ) > "$OUT/$st.log" 2>&1 || { tail -20 "$OUT/$st.log"; exit 6; }
      mkdir -p "$OUT/$st"
      python3 benchmarks/trace_window_stats.py "/tmp/$st/k_kernel_trace.csv" "$OUT/$st/steady_kernel_stats.csv" \
        >> "$OUT/$st.log" 2>&1 || exit 7
      python3 benchmarks/trace_dispatches.py "/tmp/$st/k_kernel_trace.csv" "$OUT/$st/sequence.csv" "" \
        >> "$OUT/$st.log" 2>&1 || exit 7
      python3 benchmarks/rocprof_summary.py "$OUT/$st/steady_kernel_stats.csv" "$m $prec steady state (10 steps)" 45 10 \
        > "$OUT/$st.md" || exit 7
      tail -n 3 "$OUT/$st.log" ;;
    profset:*)  # profset:MODULE:ATTR=VALUE:MODEL[-fp32] -- prof-MODEL with one module switch set
      spec=${step#profset:}
      IFS=: read -r mod kv m <<< "$spec"
      prec=bf16-amp
      if [[ $m == *-fp32 ]]; then m=${m%-fp32}; prec=fp32; fi
      R=$PWD
      st="profset-$m-${kv//=/-}$SUFFIX"
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/$st" -o k -- \
          python3 "$R/benchmarks/model_step.py" --model "$m" --steps 10 --warmup 6 --precision "$prec" \
          --profile-marker --set "$mod:$kv" ) > "$OUT/$st.log" 2>&1 || { tail -20 "$OUT/$st.log"; exit 6; }
      mkdir -p "$OUT/$st"
      python3 benchmarks/trace_window_stats.py "/tmp/$st/k_kernel_trace.csv" "$OUT/$st/steady_kernel_stats.csv" \
        >> "$OUT/$st.log" 2>&1 || exit 7
      python3 benchmarks/trace_dispatches.py "/tmp/$st/k_kernel_trace.csv" "$OUT/$st/sequence.csv" "" \
        >> "$OUT/$st.log" 2>&1 || exit 7
      python3 benchmarks/rocprof_summary.py "$OUT/$st/steady_kernel_stats.csv" "$m $prec $mod:$kv (10 steps)" 60 10 \
        > "$OUT/$st.md" || exit 7
      tail -n 3 "$OUT/$st.log" ;;
    pmc-*)
      spec=${step#pmc-}
      m=${spec%%:*}
      ctr=${spec#*:}
      run 180 "pmc-$m" rocprofv3 --kernel-trace --pmc ${ctr//,/ } -d "$OUT/pmc-$m$SUFFIX" -o run \
        --output-format csv -- python -u benchmarks/model_step.py --model "$m" --steps 3 --warmup 3 || exit $? ;;
    pytest:*)  # pytest:tests/FILE.py[,-k,EXPR] -- one GPU test file
      spec=${step#pytest:}
      run 300 "pytest-$(basename "${spec%%,*}" .py)" python -u -m pytest ${spec//,/ } -m gpu -x -q --timeout 120 \
        --timeout-method thread || exit $? ;;
    env:*)  # env:NAME=VALUE -- exported for the steps that follow
      kv=${step#env:}
      export "${kv?}"
      SUFFIX="$SUFFIX+$kv"
      echo "[lease] export $kv" ;;
    py:*)
      spec=${step#py:}
      script=${spec%%:*}
      args=""
      [[ $spec == *:* ]] && args=${spec#*:}
      run 600 "py-${script%.py}" python -u "benchmarks/$script" ${args//,/ } || exit $? ;;
    ab:*)
      spec=${step#ab:}
      IFS=: read -r name m reps <<< "$spec"
      prec=bf16-amp
      if [[ $m == *-fp32 ]]; then m=${m%-fp32}; prec=fp32; fi
      jl="$OUT/ab-$name-$m.jsonl"
      for ((i = 1; i <= ${reps:-2}; i++)); do
        for v in 1 0; do
          env "$name=$v" timeout -k 10 300 python -u benchmarks/model_step.py --model "$m" --steps 30 --warmup 10 \
            --precision "$prec" > "$OUT/ab-$name-$v-$i.log" 2>&1 || { tail -20 "$OUT/ab-$name-$v-$i.log"; exit 1; }
          echo "{\"$name\": $v, \"rep\": $i, \"run\": $(grep '^{' "$OUT/ab-$name-$v-$i.log" | tail -1)}" >> "$jl"
          tail -n 1 "$jl" | cut -c1-200
        done
      done ;;
    abset:*)
      spec=${step#abset:}
      IFS=: read -r mod attr m reps <<< "$spec"
      prec=bf16-amp
      if [[ $m == *-fp32 ]]; then m=${m%-fp32}; prec=fp32; fi
      jl="$OUT/ab-$attr-$m.jsonl"
      for ((i = 1; i <= ${reps:-2}; i++)); do
        for v in True False; do
          timeout -k 10 300 python -u benchmarks/model_step.py --model "$m" --steps 30 --warmup 10 \
            --precision "$prec" --set "$mod:$attr=$v" > "$OUT/ab-$attr-$v-$i.log" 2>&1 \
            || { tail -20 "$OUT/ab-$attr-$v-$i.log"; exit 1; }
          echo "{\"$attr\": \"$v\", \"rep\": $i, \"run\": $(grep '^{' "$OUT/ab-$attr-$v-$i.log" | tail -1)}" >> "$jl"
          tail -n 1 "$jl" | cut -c1-200
        done
      done ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[lease $(date +%T)] all steps ok"
