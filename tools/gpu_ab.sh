#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.log
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "gibbs or graph or resume" --durations=5 > gpurun_out/pytest_gibbs.log 2>&1 || { echo "pytest failed" >> gpurun_out/progress.log; exit 1; }
echo "pytest ok $(date)" >> gpurun_out/progress.log
timeout -k 10 600 python bench/gibbs_ab.py --rounds 5 --sweeps 20 > gpurun_out/gibbs_ab.json 2> gpurun_out/gibbs_ab.err || { echo "ab failed" >> gpurun_out/progress.log; exit 1; }
echo "ab ok $(date)" >> gpurun_out/progress.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed" >> gpurun_out/progress.log; exit 1; }
echo "bench ok $(date)" >> gpurun_out/progress.log
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc -o ab -- python bench/gibbs_ab.py --rounds 1 --sweeps 2 --burn 2 > gpurun_out/pmc.log 2>&1 || { echo "pmc failed" >> gpurun_out/progress.log; exit 1; }
echo "pmc ok $(date)" >> gpurun_out/progress.log
