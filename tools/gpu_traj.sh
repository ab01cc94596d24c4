#!/bin/bash
# GPU tests -> per-sweep trajectory (time + change fraction per mode) -> steady-state A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.log
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 200 > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed" >> gpurun_out/progress.log; exit 1; }
echo "pytest ok $(date)" >> gpurun_out/progress.log
timeout -k 10 600 python bench/gibbs_traj.py --sweeps 60 --modes ${TRAJ_MODES:-recount,dual,recount+lds,dual+lds} > gpurun_out/gibbs_traj.json 2> gpurun_out/gibbs_traj.err || { echo "traj failed" >> gpurun_out/progress.log; exit 1; }
echo "traj ok $(date)" >> gpurun_out/progress.log
timeout -k 10 600 python bench/gibbs_ab.py --rounds 5 --sweeps 20 --modes ${AB_MODES:-dual+qpf,dual+lds,recount+lds} > gpurun_out/gibbs_ab.json 2> gpurun_out/gibbs_ab.err || { echo "ab failed" >> gpurun_out/progress.log; exit 1; }
echo "ab ok $(date)" >> gpurun_out/progress.log
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed" >> gpurun_out/progress.log; exit 1; }
  echo "bench ok $(date)" >> gpurun_out/progress.log
fi
if [ -n "$BENCH_SRC" ]; then
  for src in $BENCH_SRC; do
    timeout -k 10 500 python bench.py --source $src --steps 30 --warmup 10 > gpurun_out/bench_$src.json 2> gpurun_out/bench_$src.err || { echo "bench $src failed" >> gpurun_out/progress.log; exit 1; }
    echo "bench $src ok $(date)" >> gpurun_out/progress.log
  done
fi
