#!/bin/bash
# multi-lane LDS sampler: kernel tests (bitwise vs fma oracle) + K=50/100 A/B against the register samplers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bitwise" \
  > gpurun_out/ldsg_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ldsg_tests.log; exit 1; }
tail -2 gpurun_out/ldsg_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gibbs_stat.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/ldsg_stat.log 2>&1 || { echo "stat tests failed"; tail -30 gpurun_out/ldsg_stat.log; exit 1; }
tail -2 gpurun_out/ldsg_stat.log
for K in 100 50; do
  timeout -k 10 300 python bench/gibbs_ab.py --topics $K --rounds 3 --sweeps 10 --burn 10 \
    --modes ${MODES:-recount,recount+lds,recount+ldsq,wdelta+lds,wdelta+ldsq} > gpurun_out/ldsg_ab_k$K.json 2> gpurun_out/ldsg_ab_k$K.err \
    || { echo "ab K=$K failed"; tail -20 gpurun_out/ldsg_ab_k$K.err; exit 1; }
  echo "ab K=$K ok"
done
