set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3zk; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 python bench.py --topics 100 --steps 3 --warmup 1 --realistic-steps 0 > $O/bench_k100.json 2> $O/bench_k100.err
