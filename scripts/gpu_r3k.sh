set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 python -u bench/gibbs_ab.py --topics 100 --modes wdelta+lds,wdelta+lds5,recount+lds,recount+lds5 --rounds 5 --sweeps 20 > $O/ab_lds5_k100.json 2> $O/ab_lds5_k100.err &&
timeout -k 10 400 python -u tools/doc_sparsity.py flow dns proxy > $O/sparsity.jsonl 2> $O/sparsity.err &&
timeout -k 10 300 python -u tools/score_anatomy.py 12500000 cuda > $O/anatomy_wide.txt 2> $O/anatomy_wide.err &&
timeout -k 10 900 python -u bench/combined.py --mode day --flows-per-gpu 62500000 --dns-per-gpu 31250000 --proxy-per-gpu 31250000 --steps 1 --warmup 1 > $O/combined_day_125M.json 2> $O/combined_day_125M.err &&
timeout -k 10 300 python -u bench/gibbs_ab.py --topics 50 --flows 1000000 --modes recount+lds,recount+lds5 --rounds 5 --sweeps 20 > $O/ab_lds5_k50.json 2> $O/ab_lds5_k50.err
