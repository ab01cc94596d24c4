set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ws or word_sparse or multilane or widen" > $O/pytest_ws.log 2>&1 &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 100 --burn 100 --modes wdelta+lds,wdelta+ws --rounds 5 --sweeps 20 > $O/ab_ws_k100.json 2> $O/ab_ws_k100.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 20 --burn 100 --modes wdelta+qpf,wdelta+ws --rounds 5 --sweeps 20 > $O/ab_ws_k20.json 2> $O/ab_ws_k20.err
