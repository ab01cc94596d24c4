#!/bin/bash
# SQ counters of the multi-lane samplers at K=100 (register "plain" vs LDS-count) — own run, --pmc only
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU \
  -d "$R/gpurun_out/pmc_k100" -o sq -- python "$R/bench/gibbs_ab.py" --topics ${K:-100} --rounds 1 --sweeps 2 --burn 2 \
  --modes recount+plain,recount+lds > "$R/gpurun_out/pmc_k100.log" 2>&1 || { echo "pmc failed"; tail -20 "$R/gpurun_out/pmc_k100.log"; exit 1; }
echo pmc ok
