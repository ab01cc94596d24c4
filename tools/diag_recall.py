"""Planted-anomaly recall of the DNS / proxy / flow pipelines vs day size (top-3000 results)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oni355.pipeline.dns import run_dns  # noqa: E402
from oni355.synth.dns import generate_dns  # noqa: E402

dev = sys.argv[1] if len(sys.argv) > 1 else "cuda"
from oni355.pipeline.proxy import run_proxy  # noqa: E402
from oni355.synth.dns import top_domain_list  # noqa: E402
from oni355.synth.proxy import generate_proxy  # noqa: E402

for src in ("dns", "proxy"):
  for n in (100_000, 2_000_000):
    for sweeps in (60,):
        if src == "dns":
            day = generate_dns(n, seed=7, n_clients=max(32, n // 40))
            res = run_dns(day.cols, K=50, sweeps=sweeps, maxresults=3000, device=dev, top_domains=day.top_domains,
                          user_domain="intel")
        else:
            day = generate_proxy(n, seed=7, n_clients=max(32, n // 40))
            res = run_proxy(day.cols, K=50, sweeps=sweeps, maxresults=3000, device=dev,
                            top_domains=top_domain_list())
            hit = np.isin(day.anomaly_rows, res.rows)
            pos = {int(r): i for i, r in enumerate(res.rows)}
            ranks = sorted(pos[int(a)] for a in day.anomaly_rows if int(a) in pos)
            print(f"{src} n={n} sweeps={sweeps} anomalies={day.anomaly_rows.size} hit={int(hit.sum())} ranks={ranks[:10]}",
                  flush=True)
