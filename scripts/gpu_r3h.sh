set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 300 python bench.py --steps 10 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 1000 python -u bench/recall_sweep.py > $O/recall.jsonl 2> $O/recall.err
