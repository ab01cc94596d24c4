set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3p; mkdir -p $O
timeout -k 10 400 python -u bench/gibbs_ab.py --topics 100 --burn 100 --modes recount+lds,dual+lds,delta+lds,wdelta+lds,atomic+lds --rounds 5 --sweeps 20 > $O/ab_modes_k100.json 2> $O/ab_modes_k100.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 50 --flows 2000000 --burn 100 --modes recount+lds,dual+lds,delta+lds,wdelta+lds --rounds 5 --sweeps 20 > $O/ab_modes_k50.json 2> $O/ab_modes_k50.err &&
Q=gpurun_out/r3q && mkdir -p $Q && R=$GRAFT_REPO_ROOT &&
timeout -k 10 300 python bench.py --steps 10 --realistic-steps 0 > $Q/bench_w1.json 2> $Q/bench_w1.err &&
ONI_FORCE_DIST=1 timeout -k 10 300 python bench.py --steps 10 --realistic-steps 0 > $Q/bench_fdp1.json 2> $Q/bench_fdp1.err &&
cd /tmp && ONI_FORCE_DIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$Q/prof_fdp1 -o fdp1 -- python3 $R/bench.py --steps 3 --warmup 1 --realistic-steps 0 > $R/$Q/prof_fdp1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$Q/prof_w1 -o w1 -- python3 $R/bench.py --steps 3 --warmup 1 --realistic-steps 0 > $R/$Q/prof_w1.log 2>&1
