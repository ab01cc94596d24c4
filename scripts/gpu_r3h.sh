set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 700 python -u bench/recall_sweep.py > $O/recall.jsonl 2> $O/recall.err
