#!/bin/bash
# K=20 one-lane LDS sampler (now with wdelta) vs the register sampler
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bitwise or graph or resume" \
  > gpurun_out/lds20_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lds20_tests.log; exit 1; }
tail -1 gpurun_out/lds20_tests.log
timeout -k 10 300 python bench/gibbs_ab.py --topics 20 --rounds 3 --sweeps 10 --burn 30 \
  --modes recount+qpf,recount+lds,wdelta+qpf,wdelta+lds > gpurun_out/lds20_ab.json 2> gpurun_out/lds20_ab.err \
  || { echo "ab failed"; tail -20 gpurun_out/lds20_ab.err; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/lds20_bench_qpf.json 2> gpurun_out/lds20_bench.err && \
ONI_SAMPLER=lds timeout -k 10 300 python bench.py > gpurun_out/lds20_bench_lds.json 2>> gpurun_out/lds20_bench.err
