#!/bin/bash
# LDS-count sampler: GPU bitwise tests -> interleaved A/B (+chunk-length sweep) -> bench -> bench profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.log
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_strings.py -x -v -m gpu --timeout 200 --durations=5 > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed" >> gpurun_out/progress.log; exit 1; }
echo "pytest ok $(date)" >> gpurun_out/progress.log
timeout -k 10 600 python bench/gibbs_ab.py --rounds 5 --sweeps 20 --modes dual+qpf,dual+lds --chunk-lens 64,128,256 --lds > gpurun_out/gibbs_ab.json 2> gpurun_out/gibbs_ab.err || { echo "ab failed" >> gpurun_out/progress.log; exit 1; }
echo "ab ok $(date)" >> gpurun_out/progress.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed" >> gpurun_out/progress.log; exit 1; }
echo "bench ok $(date)" >> gpurun_out/progress.log
ONI_SAMPLER=lds timeout -k 10 400 python bench.py > gpurun_out/bench_lds.json 2> gpurun_out/bench_lds.err || { echo "bench lds failed" >> gpurun_out/progress.log; exit 1; }
echo "bench lds ok $(date)" >> gpurun_out/progress.log
cd /tmp && ONI_SAMPLER=lds timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench_lds" -o bench -- python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 4 > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench_lds.log" 2>&1 || { echo "prof failed" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.log"; exit 1; }
echo "prof ok $(date)" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.log"
cd "$GRAFT_REPO_ROOT" && bash tools/gpu_pmc.sh >> gpurun_out/progress.log 2>&1
