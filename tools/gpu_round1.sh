#!/bin/bash
# First GPU validation: kernel tests, small + default bench, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.log
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?" >> gpurun_out/progress.log; exit 1; }
echo "pytest ok $(date)" >> gpurun_out/progress.log
timeout -k 10 600 python bench.py --flows-per-gpu 1000000 --steps 20 --warmup 5 > gpurun_out/bench_1m.json 2> gpurun_out/bench_1m.err || { echo "bench1m failed rc=$?" >> gpurun_out/progress.log; exit 1; }
echo "bench1m ok $(date)" >> gpurun_out/progress.log
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?" >> gpurun_out/progress.log; exit 1; }
echo "bench ok $(date)" >> gpurun_out/progress.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/prof.log 2>&1 || { echo "prof failed rc=$?" >> gpurun_out/progress.log; exit 1; }
echo "prof ok $(date)" >> gpurun_out/progress.log
