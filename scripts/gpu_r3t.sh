set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3t; mkdir -p $O; R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_strings.py tests/test_gpu_dist.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --realistic-steps 0 > $O/bench_w1.json 2> $O/bench_w1.err &&
timeout -k 10 300 python bench.py --source dns --steps 10 --realistic-steps 0 > $O/bench_dns.json 2> $O/bench_dns.err &&
timeout -k 10 300 python bench.py --source proxy --steps 10 --realistic-steps 0 > $O/bench_proxy.json 2> $O/bench_proxy.err &&
PROFILE_LINES=60 timeout -k 10 300 python tools/profile_host.py flow 12500000 > $O/host_profile_flow.txt 2>&1 &&
ONI_FORCE_DIST=1 timeout -k 10 300 python bench.py --steps 10 --realistic-steps 0 > $O/bench_fdp1.json 2> $O/bench_fdp1.err &&
ONI_FORCE_DIST=1 PROFILE_LINES=60 timeout -k 10 300 python tools/profile_host.py flow 12500000 > $O/host_profile_flow_fdp1.txt 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_w1 -o w1 -- python3 $R/bench.py --steps 3 --warmup 1 --realistic-steps 0 > $R/$O/prof_w1.log 2>&1
