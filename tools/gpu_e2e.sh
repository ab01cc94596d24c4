#!/bin/bash
# End-to-end on the GPU: the demo (ingest → oni-ml flow/dns/proxy → oni-oa → feedback → re-run),
# config 2 (1M synthetic flows, K=20, 200 sweeps) through the oni-ml CLI, DNS chunk-length sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/e2e
P="$R/gpurun_out/progress.log"
echo "start $(date)" > "$P"
timeout -k 10 600 bash scripts/demo.sh /tmp/oni_demo > gpurun_out/e2e/demo.log 2>&1 || { echo "demo failed rc=$?" >> "$P"; exit 1; }
cp -r /tmp/oni_demo/lp gpurun_out/e2e/demo_lp
echo "demo ok $(date)" >> "$P"
timeout -k 10 600 python -m oni355.cli.ml 20160708 flow 1.0 3000 --synthetic 1000000 --sweeps 200 --eval-every 50 \
  --lpath /tmp/oni_c2 > gpurun_out/e2e/config2.json 2> gpurun_out/e2e/config2.err || { echo "config2 failed rc=$?" >> "$P"; exit 1; }
cp /tmp/oni_c2/flow/20160708/metrics.jsonl gpurun_out/e2e/config2_metrics.jsonl
head -20 /tmp/oni_c2/flow/20160708/flow_results.csv > gpurun_out/e2e/config2_results_head.csv
echo "config2 ok $(date)" >> "$P"
for L in 8 16 32; do
  timeout -k 10 300 python bench.py --source dns --chunk-len $L > gpurun_out/e2e/dns_L$L.json 2> gpurun_out/e2e/dns_L$L.err \
    || { echo "dns L=$L failed rc=$?" >> "$P"; exit 1; }
  echo "dns L=$L ok $(date)" >> "$P"
done
