set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3u; mkdir -p $O; R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err &&
ONI_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 4 --steps 3 --warmup 1 --realistic-steps 0 > $O/bench_4ranks_gloo.json 2> $O/bench_4ranks_gloo.err &&
timeout -k 10 300 python bench.py --topics 100 --steps 3 --warmup 1 --realistic-steps 0 > $O/bench_k100.json 2> $O/bench_k100.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_w1 -o w1 -- python3 $R/bench.py --steps 3 --warmup 1 --realistic-steps 0 > $R/$O/prof_w1.log 2>&1
