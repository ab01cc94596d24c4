#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.log
timeout -k 10 700 python -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 120 --durations=0 -k "gibbs or graph or resume" > gpurun_out/pytest_diag.log 2>&1 || { echo "pytest failed" >> gpurun_out/progress.log; exit 1; }
echo "pytest ok $(date)" >> gpurun_out/progress.log
timeout -k 10 400 python bench/gibbs_ab.py --rounds 5 --sweeps 20 > gpurun_out/gibbs_ab.json 2> gpurun_out/gibbs_ab.err || { echo "ab failed" >> gpurun_out/progress.log; exit 1; }
echo "ab ok $(date)" >> gpurun_out/progress.log
