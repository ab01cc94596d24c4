#!/bin/bash
# kernel trace of the first 30 sweeps (per-dispatch durations: which kernel slows down early on)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_traj" -o tt -- python "$R/bench/gibbs_traj.py" --sweeps 30 --modes ${TRAJ_MODES:-recount} > "$R/gpurun_out/trace_traj.log" 2>&1 || { echo "trace failed"; exit 1; }
echo trace ok
