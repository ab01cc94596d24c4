set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3za; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "q2" > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench/gibbs_ab.py --topics 20 --burn 30 --modes recount+qpf,recount+q2,wdelta+qpf,wdelta+q2,recount+pp > $O/ab_k20_burn30.json 2> $O/ab_k20_burn30.err &&
timeout -k 10 600 python -u bench/gibbs_ab.py --topics 20 --burn 150 --modes recount+qpf,recount+q2,wdelta+qpf,wdelta+q2 > $O/ab_k20_burn150.json 2> $O/ab_k20_burn150.err
