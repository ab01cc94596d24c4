set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3zg; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gibbs_stat.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench/gibbs_ab.py --topics 20 --burn 150 --modes recount+qpf,recount+lds,wdelta+q2,wdelta+lds > $O/ab_k20_burn150.json 2> $O/ab_k20_burn150.err &&
timeout -k 10 600 python -u bench/gibbs_ab.py --topics 20 --burn 10 --modes recount+qpf,recount+lds,wdelta+q2,wdelta+lds > $O/ab_k20_burn10.json 2> $O/ab_k20_burn10.err
