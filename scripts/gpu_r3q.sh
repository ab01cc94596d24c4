set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3q; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 10 --realistic-steps 0 > $O/bench_w1.json 2> $O/bench_w1.err &&
ONI_FORCE_DIST=1 timeout -k 10 300 python bench.py --steps 10 --realistic-steps 0 > $O/bench_fdp1.json 2> $O/bench_fdp1.err &&
cd /tmp && ONI_FORCE_DIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_fdp1 -o fdp1 -- python3 $R/bench.py --steps 3 --warmup 1 --realistic-steps 0 > $R/$O/prof_fdp1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_w1 -o w1 -- python3 $R/bench.py --steps 3 --warmup 1 --realistic-steps 0 > $R/$O/prof_w1.log 2>&1
