set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3zj; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench/gibbs_ab.py --topics 20 --burn 150 --modes recount+qpf,wdelta+qpf,wdelta+q2 > $O/ab_k20_burn150.json 2> $O/ab_k20_burn150.err &&
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
