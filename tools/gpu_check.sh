#!/bin/bash
# Round-end rehearsal: GPU test-suite, smoke(), default bench (N=1), kernel stats of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P="$R/gpurun_out/progress.log"
echo "start $(date)" > "$P"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?" >> "$P"; exit 1; }
echo "pytest ok $(date)" >> "$P"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { echo "smoke failed rc=$?" >> "$P"; exit 1; }
echo "smoke ok $(date)" >> "$P"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { echo "bench failed rc=$?" >> "$P"; exit 1; }
echo "bench ok $(date)" >> "$P"
if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
    -- python "$R/bench.py" --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$R/gpurun_out/prof.log" 2>&1 \
    || { echo "prof failed rc=$?" >> "$P"; exit 1; }
  echo "prof ok $(date)" >> "$P"
fi
