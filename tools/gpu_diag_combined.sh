#!/bin/bash
# locate the combined-bench setup stall: small sizes first, then the real shard
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
DIAG_FLOWS=1000000 DIAG_DNS=500000 timeout -k 10 150 python tools/diag_combined.py > gpurun_out/diag_small.log 2>&1 \
  && DIAG_FLOWS=0 timeout -k 10 150 python tools/diag_combined.py > gpurun_out/diag_dns_only.log 2>&1 \
  && timeout -k 10 200 python tools/diag_combined.py > gpurun_out/diag_full.log 2>&1
