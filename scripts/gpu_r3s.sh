set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3s; mkdir -p $O; R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --realistic-steps 0 > $O/bench_w1.json 2> $O/bench_w1.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_w1 -o w1 -- python3 $R/bench.py --steps 3 --warmup 1 --realistic-steps 0 > $R/$O/prof_w1.log 2>&1 &&
cd $R && O2=gpurun_out/r3r && mkdir -p $O2 &&
timeout -k 10 300 python bench.py --realistic-vocab --lt-codebook 0.04 --steps 3 --warmup 1 --realistic-steps 0 > $O2/bench_wide459k.json 2> $O2/bench_wide459k.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --wide --lt-codebook 0.04 --burn 100 --modes wdelta+qpf,wdelta+q2,wdelta+dz --rounds 5 --sweeps 20 > $O2/ab_wide459k.json 2> $O2/ab_wide459k.err &&
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O2/pmc_fetch -o f -- python3 $R/bench/gibbs_ab.py --wide --lt-codebook 0.04 --burn 100 --modes wdelta+qpf --rounds 1 --sweeps 5 > $R/$O2/pmc_fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/$O2/pmc_tcc -o t -- python3 $R/bench/gibbs_ab.py --wide --lt-codebook 0.04 --burn 100 --modes wdelta+qpf --rounds 1 --sweeps 5 > $R/$O2/pmc_tcc.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O2/pmc_fetch_narrow -o f -- python3 $R/bench/gibbs_ab.py --burn 100 --modes wdelta+qpf --rounds 1 --sweeps 5 > $R/$O2/pmc_fetch_narrow.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/$O2/pmc_tcc_narrow -o t -- python3 $R/bench/gibbs_ab.py --burn 100 --modes wdelta+qpf --rounds 1 --sweeps 5 > $R/$O2/pmc_tcc_narrow.log 2>&1
