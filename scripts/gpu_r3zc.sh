set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3zc; mkdir -p $O
timeout -k 10 600 python -u bench/gibbs_ab.py --topics 100 --burn 100 --modes recount+lds,recount+ldsq,wdelta+lds,wdelta+ldsq > $O/ab_k100.json 2> $O/ab_k100.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 50 --burn 100 --modes recount+lds,recount+ldsq,wdelta+lds,wdelta+ldsq > $O/ab_k50.json 2> $O/ab_k50.err
