set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3r; mkdir -p $O; R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --realistic-vocab --lt-codebook 0.04 --steps 3 --warmup 1 --realistic-steps 0 > $O/bench_wide459k.json 2> $O/bench_wide459k.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --wide --lt-codebook 0.04 --burn 100 --modes wdelta+qpf,wdelta+q2,wdelta+dz --rounds 5 --sweeps 20 > $O/ab_wide459k.json 2> $O/ab_wide459k.err &&
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o f -- python3 $R/bench/gibbs_ab.py --wide --lt-codebook 0.04 --burn 100 --modes wdelta+qpf --rounds 1 --sweeps 5 > $R/$O/pmc_fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/$O/pmc_tcc -o t -- python3 $R/bench/gibbs_ab.py --wide --lt-codebook 0.04 --burn 100 --modes wdelta+qpf --rounds 1 --sweeps 5 > $R/$O/pmc_tcc.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch_narrow -o f -- python3 $R/bench/gibbs_ab.py --burn 100 --modes wdelta+qpf --rounds 1 --sweeps 5 > $R/$O/pmc_fetch_narrow.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/$O/pmc_tcc_narrow -o t -- python3 $R/bench/gibbs_ab.py --burn 100 --modes wdelta+qpf --rounds 1 --sweeps 5 > $R/$O/pmc_tcc_narrow.log 2>&1
