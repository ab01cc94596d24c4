set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3zh; mkdir -p $O
for t in 0.12 0.3 0.6 1.0; do
  ONI_AUTO_THRESHOLD=$t timeout -k 10 300 python bench.py --realistic-steps 0 > $O/bench_thr_$t.json 2> $O/bench_thr_$t.err || exit 1
done
