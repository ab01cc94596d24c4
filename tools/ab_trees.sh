#!/bin/bash
# A/B of two trees' default day on ONE box (alternating runs): the current tree and a side
# worktree ab_old/ of another commit (git worktree add ab_old <commit>; python tools/build.py inside it).
# Usage: bash tools/ab_trees.sh TAG REPS [bench args]
set -o pipefail
TOP="$(cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && pwd)"
[[ "${STAGE:-0}" == "1" ]] && SRC="$TOP/gpurun_stage" || SRC="$TOP"
OUT="$TOP/gpurun_out/$1"; mkdir -p "$OUT"
reps="$2"; shift 2
for r in $(seq 1 "$reps"); do
  for t in old new; do
    d="$SRC"; [[ "$t" == "old" ]] && d="$SRC/ab_old"
    (cd "$d" && timeout -k 10 300 python -u bench.py "$@" > "$OUT/${t}_$r.json" 2> "$OUT/${t}_$r.err") || exit $?
    echo "$(date +%T) $t $r $(python -c "import json;d=json.load(open('$OUT/${t}_$r.json'));print(d['ms_per_step'],d['ms_per_sweep_in_training'])")" | tee -a "$OUT/progress.log"
  done
done
