#!/bin/bash
# config 5: combined flow+dns+proxy, K=100 — default shard, then one GPU's share of the 1B-event day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P="gpurun_out/progress.log"
echo "start $(date)" > "$P"
timeout -k 10 300 python bench/combined.py > gpurun_out/combined_25M.json 2> gpurun_out/combined_25M.err \
  || { echo "combined 25M failed rc=$?" >> "$P"; exit 1; }
echo "combined 25M ok $(date)" >> "$P"
timeout -k 10 600 python bench/combined.py --flows-per-gpu 62500000 --dns-per-gpu 31250000 --proxy-per-gpu 31250000 \
  --steps 10 --warmup 5 > gpurun_out/combined_125M.json 2> gpurun_out/combined_125M.err \
  || { echo "combined 125M failed rc=$?" >> "$P"; exit 1; }
echo "combined 125M ok $(date)" >> "$P"
