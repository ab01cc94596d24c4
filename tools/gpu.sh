#!/bin/bash
# One parameterised GPU runner for gpurun (replaces the round-1 one-off scripts).
#
#   gpurun --timeout 1200 -- bash tools/gpu.sh STEP [STEP ...]
#
# Every STEP runs under its own `timeout -k 10`, writes its output under gpurun_out/<tag>/ and the
# chain stops at the first failure (no retries: a fault/abort/timeout ends the call).
#   tests                 python -m pytest -m gpu (all GPU tests, one process)
#   tests:<file>          one test file
#   smoke                 __graft_entry__.smoke()
#   bench[:<args>]        python bench.py <args>            (args: comma-separated, e.g. bench:--steps,20)
#   prof[:<args>]         rocprofv3 --kernel-trace --stats -- python bench.py <args>
#   mprof[:<args>]        the same plus --marker-trace (the package's roctx ranges)
#   pmc:<ctrs>[:<args>]   rocprofv3 --pmc <ctrs> --kernel-trace --stats (ctrs comma-separated)
#   py:<script>[:<args>]  python <script> <args>
#   list                  rocprofv3 --list-avail (PMC counter names of this GPU)
# TAG env var (default "run") names the output directory.
# STAGE=1: run the frozen copy in gpurun_stage/ (tools/stage.sh made it while the tree was consistent)
# so that edits made while the call waits for a box cannot mix into it; output still goes to the
# top-level gpurun_out/.
set -o pipefail
TOP="$(cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && pwd)"
cd "$TOP"
[[ "${STAGE:-0}" == "1" ]] && cd "$TOP/gpurun_stage"
export TMPDIR=/tmp
TAG="${TAG:-run}"
OUT="$TOP/gpurun_out/$TAG"
mkdir -p "$OUT"
log() { echo "$(date +%T) $*" | tee -a "$OUT/progress.log"; }
n=0
for step in "$@"; do
  n=$((n + 1))
  kind="${step%%:*}"
  rest=""
  [[ "$step" == *:* ]] && rest="${step#*:}"
  log "step $n: $step"
  case "$kind" in
    tests)
      tgt="tests"; [[ -n "$rest" ]] && tgt="$rest"
      timeout -k 10 1000 python -u -m pytest "$tgt" -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_$n.log" 2>&1; rc=$? ;;
    smoke)
      timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke_$n.log" 2>&1; rc=$? ;;
    bench)
      IFS=',' read -r -a args <<< "$rest"
      timeout -k 10 900 python -u bench.py "${args[@]}" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err"; rc=$? ;;
    prof)
      IFS=',' read -r -a args <<< "$rest"
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$n" -o run \
        -- python3 -u bench.py "${args[@]}" > "$OUT/prof_$n.log" 2>&1; rc=$? ;;
    mprof)
      IFS=',' read -r -a args <<< "$rest"
      timeout -k 10 900 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d "$OUT/mprof_$n" -o run \
        -- python3 -u bench.py "${args[@]}" > "$OUT/mprof_$n.log" 2>&1; rc=$? ;;
    pmc)
      ctrs="${rest%%:*}"; bargs=""; [[ "$rest" == *:* ]] && bargs="${rest#*:}"
      IFS=',' read -r -a args <<< "$bargs"
      timeout -s KILL 300 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace --stats --output-format csv -d "$OUT/pmc_$n" -o run \
        -- python3 -u bench.py "${args[@]}" > "$OUT/pmc_$n.log" 2>&1; rc=$? ;;
    list)
      timeout -k 10 120 rocprofv3 --list-avail > "$OUT/counters_$n.txt" 2>&1; rc=$? ;;
    py)
      script="${rest%%:*}"; pargs=""; [[ "$rest" == *:* ]] && pargs="${rest#*:}"
      IFS=',' read -r -a args <<< "$pargs"
      timeout -k 10 900 python -u "$script" "${args[@]}" > "$OUT/py_$n.log" 2>&1; rc=$? ;;
    *) log "unknown step $kind"; exit 2 ;;
  esac
  log "step $n rc=$rc"
  if [[ $rc -ne 0 ]]; then exit $rc; fi
done
log "all steps ok"
