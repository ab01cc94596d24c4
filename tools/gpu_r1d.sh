#!/bin/bash
# q-prefetch sampler for multi-lane units (K=50): tests + DNS/proxy A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P="$R/gpurun_out/progress.log"
echo "start $(date)" > "$P"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?" >> "$P"; exit 1; }
echo "pytest ok $(date)" >> "$P"
for src in dns proxy; do
  for smp in plain qpf pp; do
    ONI_SAMPLER=$smp timeout -k 10 300 python bench.py --source $src > gpurun_out/b_${src}_$smp.json 2> gpurun_out/b_${src}_$smp.err \
      || { echo "bench $src $smp failed rc=$?" >> "$P"; exit 1; }
    echo "bench $src $smp ok $(date)" >> "$P"
  done
done
