set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3ze; mkdir -p $O; R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o day -- python3 $R/bench.py --steps 3 --warmup 1 --realistic-steps 0 > $R/$O/prof.log 2>&1
