#!/bin/bash
# End-to-end demo (the oni-demo container equivalent):
# synthetic day → ingest → oni-ml (flow, dns, proxy) → oni-oa enrich → analyst feedback → re-run.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
WORK="${1:-/tmp/oni_demo}"
DATE=20160708
DEV="${ONI_DEVICE:-$(python -c 'import torch;print("cuda" if torch.cuda.is_available() else "cpu")')}"
rm -rf "$WORK"; mkdir -p "$WORK/collector/flow" "$WORK/collector/dns" "$WORK/collector/proxy"
cd "$ROOT"
[ -f oni355/_lib/liboni_hip.so ] && [ -f oni355/_lib/liboni_native.so ] || python tools/build.py >/dev/null
python - "$WORK" <<'PY'
import sys
from oni355.synth.flow import generate_flows
from oni355.synth.dns import generate_dns, write_pcap, top_domain_list
from oni355.synth.proxy import generate_proxy, write_log
from oni355.io.nfcapd import write_nfcapd
w = sys.argv[1]
write_nfcapd(f"{w}/collector/flow/nfcapd.201607080000", generate_flows(200_000, seed=1).cols, "lzo")
write_pcap(generate_dns(100_000, seed=2), f"{w}/collector/dns/dns_20160708.pcap")
write_log(generate_proxy(50_000, seed=3), f"{w}/collector/proxy/access_20160708.log")
open(f"{w}/top-1m.csv", "w").write("".join(f"{i+1},{d}\n" for i, d in enumerate(top_domain_list())))
PY
for t in flow dns proxy; do
  python -m oni355.cli.ingest -t $t --collector-path "$WORK/collector/$t" --data-root "$WORK/store" --once
done
K_DNS=50
python -m oni355.cli.ml $DATE flow 1.0 500 --data-root "$WORK/store" --lpath "$WORK/lp" --device $DEV --sweeps 100
python -m oni355.cli.ml $DATE dns 1.0 500 --data-root "$WORK/store" --lpath "$WORK/lp" --device $DEV --sweeps 100 \
  --topics $K_DNS --top-domains "$WORK/top-1m.csv" --user-domain intel
python -m oni355.cli.ml $DATE proxy 1.0 500 --data-root "$WORK/store" --lpath "$WORK/lp" --device $DEV --sweeps 100 \
  --top-domains "$WORK/top-1m.csv"
for t in flow dns proxy; do
  python -m oni355.cli.oa -d $DATE -t $t -l 500 --lpath "$WORK/lp"
  python -m oni355.cli.oa report -d $DATE -t $t --lpath "$WORK/lp" -l 100
done
python -m oni355.cli.oa score -d $DATE -t flow --rows 0,1,2 --sev 3 --lpath "$WORK/lp"
python -m oni355.cli.oa publish -d $DATE -t flow --lpath "$WORK/lp"
python -m oni355.cli.ml $DATE flow 1.0 500 --data-root "$WORK/store" --lpath "$WORK/lp" --device $DEV --sweeps 100
echo "demo outputs under $WORK/lp"
