#!/bin/bash
# kernel stats for the flow bench (default config) and the DNS bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_flow" -o flow -- python "$R/bench.py" > "$R/gpurun_out/prof_flow.log" 2>&1 || { echo "prof flow failed"; exit 1; }
echo "prof flow ok"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_dns" -o dns -- python "$R/bench.py" --source dns --steps 30 --warmup 10 > "$R/gpurun_out/prof_dns.log" 2>&1 || { echo "prof dns failed"; exit 1; }
echo "prof dns ok"
