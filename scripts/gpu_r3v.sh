set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3v; mkdir -p $O; R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench/cli_days.py --flows 12500000 --days 5 --cold-flows 1000000 > $O/cli_days.json 2> $O/cli_days.err &&
timeout -k 10 300 python bench.py --from-store --steps 10 --realistic-steps 0 > $O/bench_from_store.json 2> $O/bench_from_store.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_proxy -o p -- python3 $R/bench.py --source proxy --steps 3 --warmup 1 --realistic-steps 0 > $R/$O/prof_proxy.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_dns -o d -- python3 $R/bench.py --source dns --steps 3 --warmup 1 --realistic-steps 0 > $R/$O/prof_dns.log 2>&1
