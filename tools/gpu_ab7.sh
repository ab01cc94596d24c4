#!/bin/bash
# sampler variants: pp vs qpf (flow, K=20) and pp vs plain (DNS, K=50)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.log
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 200 > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed" >> gpurun_out/progress.log; exit 1; }
echo "pytest ok $(date)" >> gpurun_out/progress.log
timeout -k 10 600 python bench/gibbs_ab.py --rounds 5 --sweeps 20 --modes delta,delta+qpf,recount,recount+qpf > gpurun_out/gibbs_ab.json 2> gpurun_out/gibbs_ab.err || { echo "ab failed" >> gpurun_out/progress.log; exit 1; }
echo "ab ok $(date)" >> gpurun_out/progress.log
for smp in pp plain; do
  ONI_SAMPLER=$smp timeout -k 10 500 python bench.py --source dns --steps 30 --warmup 10 > gpurun_out/bench_dns_$smp.json 2> gpurun_out/bench_dns_$smp.err || { echo "bench dns $smp failed" >> gpurun_out/progress.log; exit 1; }
  echo "bench dns $smp ok $(date)" >> gpurun_out/progress.log
done
for smp in pp qpf; do
  ONI_SAMPLER=$smp timeout -k 10 500 python bench.py > gpurun_out/bench_$smp.json 2> gpurun_out/bench_$smp.err || { echo "bench $smp failed" >> gpurun_out/progress.log; exit 1; }
  echo "bench $smp ok $(date)" >> gpurun_out/progress.log
done
