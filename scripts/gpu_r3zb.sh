set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3zb; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 python bench.py --source dns --steps 10 --realistic-steps 0 > $O/bench_dns.json 2> $O/bench_dns.err &&
timeout -k 10 300 python bench.py --source proxy --steps 10 --realistic-steps 0 > $O/bench_proxy.json 2> $O/bench_proxy.err
