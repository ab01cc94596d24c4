#!/bin/bash
# Alternating A/B of two bench.py argument sets on ONE box: bash tools/ab_bench.sh TAG REPS "ARGS_A" "ARGS_B"
# (each run under its own time limit; the chain stops at the first failure).
set -o pipefail
TOP="$(cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && pwd)"
[[ "${STAGE:-0}" == "1" ]] && SRC="$TOP/gpurun_stage" || SRC="$TOP"
OUT="$TOP/gpurun_out/$1"; mkdir -p "$OUT"
reps="$2"; A="$3"; B="$4"
cd "$SRC"
for r in $(seq 1 "$reps"); do
  for t in A B; do
    args="$A"; [[ "$t" == "B" ]] && args="$B"
    timeout -k 10 600 python -u bench.py $args > "$OUT/${t}_$r.json" 2> "$OUT/${t}_$r.err" || exit $?
    echo "$(date +%T) $t $r $(python -c "import json;d=json.load(open('$OUT/${t}_$r.json'));print(d['ms_per_step'],d['ms_per_sweep_in_training'],d['planted_anomaly_recall_topN'])")" | tee -a "$OUT/progress.log"
  done
done
