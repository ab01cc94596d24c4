#!/bin/bash
# full GPU test suite + smoke + headline flow bench + DNS (config 3) + combined (config 5) with the current kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P=gpurun_out/progress.log
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo "pytest failed rc=$?" >> $P; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo "pytest ok $(date): $(tail -1 gpurun_out/pytest_gpu.log)" >> $P
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?" >> $P; exit 1; }
echo "smoke ok $(date)" >> $P
timeout -k 10 400 python bench.py > gpurun_out/bench_flow.json 2> gpurun_out/bench_flow.err || { echo "bench flow failed rc=$?" >> $P; exit 1; }
echo "bench flow ok $(date)" >> $P
timeout -k 10 400 python bench.py --source dns > gpurun_out/bench_dns.json 2> gpurun_out/bench_dns.err || { echo "bench dns failed rc=$?" >> $P; exit 1; }
echo "bench dns ok $(date)" >> $P
timeout -k 10 400 python bench.py --source proxy > gpurun_out/bench_proxy.json 2> gpurun_out/bench_proxy.err || { echo "bench proxy failed rc=$?" >> $P; exit 1; }
echo "bench proxy ok $(date)" >> $P
timeout -k 10 400 python bench/combined.py > gpurun_out/combined_25M.json 2> gpurun_out/combined_25M.err || { echo "combined failed rc=$?" >> $P; exit 1; }
echo "combined ok $(date)" >> $P
