#!/bin/bash
# bench + kernel stats for the DNS (config 3, K=50) and proxy sources
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P="$R/gpurun_out/progress.log"
echo "start $(date)" > "$P"
for src in dns proxy; do
  timeout -k 10 300 python bench.py --source $src > gpurun_out/bench_$src.json 2> gpurun_out/bench_$src.err \
    || { echo "bench $src failed rc=$?" >> "$P"; exit 1; }
  echo "bench $src ok $(date)" >> "$P"
done
cd /tmp && export TMPDIR=/tmp
for src in dns proxy; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$src" -o $src \
    -- python "$R/bench.py" --source $src --steps 30 --warmup 10 > "$R/gpurun_out/prof_$src.log" 2>&1 \
    || { echo "prof $src failed rc=$?" >> "$P"; exit 1; }
  echo "prof $src ok $(date)" >> "$P"
done
