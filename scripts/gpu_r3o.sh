set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3o; mkdir -p $O
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 100 --burn 100 --modes wdelta+lds,wdelta+ws,recount+lds,recount+ws,recount+ws:nostore --rounds 5 --sweeps 20 > $O/ab_ws_k100.json 2> $O/ab_ws_k100.err
