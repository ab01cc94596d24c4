set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ws or word_sparse or multilane" > $O/pytest_ws.log 2>&1 &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 100 --burn 100 --modes wdelta+lds,wdelta+ws,recount+lds,recount+ws --rounds 5 --sweeps 20 > $O/ab_ws_k100.json 2> $O/ab_ws_k100.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 20 --burn 100 --modes wdelta+qpf,wdelta+ws --rounds 5 --sweeps 20 > $O/ab_ws_k20.json 2> $O/ab_ws_k20.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 50 --burn 100 --modes wdelta+lds,wdelta+ws --rounds 5 --sweeps 20 > $O/ab_ws_k50.json 2> $O/ab_ws_k50.err &&
timeout -k 10 300 python bench.py --topics 100 --steps 3 --warmup 1 --realistic-steps 0 > $O/bench_k100_lds.json 2> $O/bench_k100_lds.err &&
ONI_SAMPLER=wsa timeout -k 10 300 python bench.py --topics 100 --steps 3 --warmup 1 --realistic-steps 0 > $O/bench_k100_wsa.json 2> $O/bench_k100_wsa.err
