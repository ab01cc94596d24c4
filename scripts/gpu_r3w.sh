set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3w; mkdir -p $O; R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_strings.py tests/test_noise_filter.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --source proxy --steps 10 --realistic-steps 0 > $O/bench_proxy.json 2> $O/bench_proxy.err &&
timeout -k 10 900 python -u bench/combined.py --mode day --flows-per-gpu 62500000 --dns-per-gpu 31250000 --proxy-per-gpu 31250000 --steps 1 --warmup 1 > $O/combined_day_125M.json 2> $O/combined_day_125M.err
