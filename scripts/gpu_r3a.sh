set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 500 python -u bench/gibbs_ab.py --modes wdelta+qpf,wdelta+q2,wdelta+q2dz,recount+qpf,recount+q2dz --rounds 7 > $O/ab.log 2>&1 &&
ONI_SAMPLER=q2dz timeout -k 10 300 python bench.py --steps 10 > $O/bench_q2dz.json 2> $O/bench_q2dz.err
