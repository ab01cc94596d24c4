#!/bin/bash
# score-kernel fixes + auto count-mode threshold sweep (bench N=1), kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P="$R/gpurun_out/progress.log"
echo "start $(date)" > "$P"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "score or tile or graph or wdelta" > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?" >> "$P"; exit 1; }
echo "pytest ok $(date)" >> "$P"
for cfg in "delta 0.08" "wdelta 0.08" "wdelta 0.12" "wdelta 0.16"; do
  set -- $cfg
  ONI_AUTO_DELTA=$1 ONI_AUTO_THRESHOLD=$2 timeout -k 10 300 python bench.py > gpurun_out/bench_$1_$2.json 2> gpurun_out/bench_$1_$2.err \
    || { echo "bench $cfg failed rc=$?" >> "$P"; exit 1; }
  echo "bench $cfg ok $(date)" >> "$P"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
  -- python "$R/bench.py" > "$R/gpurun_out/prof.log" 2>&1 || { echo "prof failed rc=$?" >> "$P"; exit 1; }
echo "prof ok $(date)" >> "$P"
