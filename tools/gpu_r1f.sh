#!/bin/bash
# shared-GPU DP tests + staging tests, then one GPU's share of the 1B-event combined day (config 5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_staging.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/dist_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/dist_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
ONI_HEARTBEAT_S=30 timeout -k 10 800 python bench/combined.py --flows-per-gpu 62500000 --dns-per-gpu 31250000 \
  --proxy-per-gpu 31250000 --steps 10 --warmup 5 > gpurun_out/combined_125M_v2.json 2> gpurun_out/combined_125M_v2.err
