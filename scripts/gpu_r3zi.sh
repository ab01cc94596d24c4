set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3zi; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pp or plain or lds or q2" > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench/gibbs_ab.py --topics 20 --burn 150 --modes recount+qpf,recount+pp,wdelta+q2,wdelta+pp > $O/ab_k20_burn150.json 2> $O/ab_k20_burn150.err
