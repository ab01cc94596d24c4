set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 300 python -u tools/score_anatomy.py 12500000 cuda > $O/anatomy_wide.txt 2> $O/anatomy_wide.err &&
timeout -k 10 600 python -u bench/combined.py --mode day > $O/combined_day.json 2> $O/combined_day.err
