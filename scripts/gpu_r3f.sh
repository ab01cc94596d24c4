set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3f; mkdir -p $O
timeout -k 10 500 python -u bench/staleness_audit.py --flows 1000000 --chunk-lens 128,128@1,1024,0 > $O/staleness_1M.jsonl 2> $O/staleness_1M.err &&
timeout -k 10 500 python -u bench/staleness_audit.py --flows 12500000 --chunk-lens 128,128@1,1024,4096 > $O/staleness_12.5M.jsonl 2> $O/staleness_12.5M.err &&
timeout -k 10 900 python -u bench/cli_days.py --flows 12500000 --days 5 > $O/cli_days.json 2> $O/cli_days.err
