set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3z2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gibbs_stat.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lds or wsg or recovers" > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench/gibbs_ab.py --topics 100 --burn 100 --modes recount+lds,wdelta+lds,recount+lds5,wdelta+lds5 > $O/ab_k100.json 2> $O/ab_k100.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 50 --burn 100 --modes recount+lds,wdelta+lds > $O/ab_k50.json 2> $O/ab_k50.err
