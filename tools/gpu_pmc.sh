#!/bin/bash
# PMC counters for the sampler variants (own run: --pmc only with --kernel-trace/--stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS \
  -d "$R/gpurun_out/pmc" -o sq -- python "$R/bench/gibbs_ab.py" --rounds 1 --sweeps 4 --burn 4 --modes ${MODES:-dual+qpf,dual+lds} > "$R/gpurun_out/pmc.log" 2>&1 || { echo "pmc failed"; exit 1; }
echo pmc ok
