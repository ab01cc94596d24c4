#!/bin/bash
# why does a 6.25M-event DNS shard take minutes to set up? periodic Python stacks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -c "
import faulthandler, sys, runpy
faulthandler.dump_traceback_later(45, repeat=True)
sys.argv = ['bench.py', '--source', 'dns', '--events-per-gpu', '6250000', '--steps', '5', '--warmup', '2']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/diag_dns.json 2> gpurun_out/diag_dns.err; echo "rc=$?" >> gpurun_out/diag_dns.err
