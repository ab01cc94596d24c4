#!/bin/bash
# config 5: kernel stats of the K=100 combined step, then one GPU's share of the 1B-event day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P="$R/gpurun_out/progress.log"
echo "start $(date)" > "$P"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/prof_comb" -o comb -- python "$R/bench/combined.py" --steps 10 --warmup 10 \
  > "$R/gpurun_out/prof_comb.log" 2>&1) || { echo "prof combined failed rc=$?" >> "$P"; exit 1; }
echo "prof combined ok $(date)" >> "$P"
timeout -k 10 700 python bench/combined.py --flows-per-gpu 62500000 --dns-per-gpu 31250000 --proxy-per-gpu 31250000 \
  --steps 10 --warmup 5 > gpurun_out/combined_125M.json 2> gpurun_out/combined_125M.err \
  || { echo "combined 125M failed rc=$?" >> "$P"; exit 1; }
echo "combined 125M ok $(date)" >> "$P"
