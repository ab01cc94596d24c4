#!/bin/bash
# MFMA scoring + word-bitmap delta recount: GPU tests, count-mode A/B, bench A/B, MFMA counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P="$R/gpurun_out/progress.log"
echo "start $(date)" > "$P"
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?" >> "$P"; exit 1; }
echo "pytest ok $(date)" >> "$P"
timeout -k 10 600 python bench/gibbs_ab.py --rounds 3 --sweeps 10 --burn 0 --modes recount,dual,delta,wdelta \
  > gpurun_out/ab_burn0.json 2> gpurun_out/ab_burn0.err || { echo "ab0 failed rc=$?" >> "$P"; exit 1; }
echo "ab0 ok $(date)" >> "$P"
timeout -k 10 600 python bench/gibbs_ab.py --rounds 3 --sweeps 10 --burn 30 --modes recount,dual,delta,wdelta \
  > gpurun_out/ab_burn30.json 2> gpurun_out/ab_burn30.err || { echo "ab30 failed rc=$?" >> "$P"; exit 1; }
echo "ab30 ok $(date)" >> "$P"
timeout -k 10 600 python bench.py > gpurun_out/bench_auto.json 2> gpurun_out/bench_auto.err \
  || { echo "bench auto failed rc=$?" >> "$P"; exit 1; }
echo "bench auto ok $(date)" >> "$P"
ONI_COUNT_MODE=wdelta timeout -k 10 600 python bench.py > gpurun_out/bench_wdelta.json 2> gpurun_out/bench_wdelta.err \
  || { echo "bench wdelta failed rc=$?" >> "$P"; exit 1; }
echo "bench wdelta ok $(date)" >> "$P"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv \
  --kernel-include-regex "k_tile_score|k_pair_score|k_event_min" \
  --pmc SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES \
  -d "$R/gpurun_out/pmc_score" -o score -- python "$R/bench.py" --steps 2 --warmup 1 \
  > "$R/gpurun_out/pmc_score.log" 2>&1 || { echo "pmc failed rc=$?" >> "$P"; exit 1; }
echo "pmc ok $(date)" >> "$P"
