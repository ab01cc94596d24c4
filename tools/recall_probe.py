#!/usr/bin/env python3
"""Planted-anomaly recall of one synthetic day (any source), default or realistic vocabulary.

  python tools/recall_probe.py --source flow --n 200000 --wide --device cpu --sweeps 100

Prints one JSON line: recall in the top-N, the rank of every planted row in the full ascending
score order (how far the misses are), the vocabulary size and how many day tokens share each
planted row's word (an anomaly whose word is common cannot be found by P(word | doc))."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--source", choices=["flow", "dns", "proxy"], default="flow")
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--wide", action="store_true")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--topics", type=int, default=None)
    ap.add_argument("--maxresults", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--chunk-len", type=int, default=0)
    ap.add_argument("--anomaly-kind", default=None, help="dns / proxy generators: rare | rare-active | offprofile")
    ap.add_argument("--lt-codebook", type=float, default=0.01, help="flow --wide: long-tail behaviours per flow")
    a = ap.parse_args()
    import numpy as np
    K = a.topics or (50 if a.source == "dns" else 20)
    t0 = time.perf_counter()
    if a.source == "flow":
        from oni355.pipeline.flow import run_flow
        from oni355.synth.flow import generate_flows
        day = generate_flows(a.n, seed=a.seed, n_hosts=max(64, a.n // 25), wide_vocab=a.wide, lt_codebook=a.lt_codebook)
        res = run_flow(day.cols, K=K, sweeps=a.sweeps, maxresults=a.n, device=a.device, chunk_len=a.chunk_len)
    elif a.source == "dns":
        from oni355.pipeline.dns import run_dns
        from oni355.synth.dns import generate_dns
        day = generate_dns(a.n, seed=a.seed, n_clients=max(32, a.n // 40), wide_vocab=0.5 if a.wide else 0.0,
                           **({"anomaly_kind": a.anomaly_kind} if a.anomaly_kind else {}))
        res = run_dns(day.cols, K=K, sweeps=a.sweeps, maxresults=a.n, device=a.device, top_domains=day.top_domains,
                      user_domain="intel", chunk_len=a.chunk_len)
    else:
        from oni355.pipeline.proxy import run_proxy
        from oni355.synth.dns import top_domain_list
        from oni355.synth.proxy import generate_proxy
        day = generate_proxy(a.n, seed=a.seed, n_clients=max(32, a.n // 40), wide_vocab=0.5 if a.wide else 0.0,
                             **({"anomaly_kind": a.anomaly_kind} if a.anomaly_kind else {}))
        res = run_proxy(day.cols, K=K, sweeps=a.sweeps, maxresults=a.n, device=a.device,
                        top_domains=top_domain_list(), chunk_len=a.chunk_len)
    rank = {int(r): i for i, r in enumerate(res.rows)}
    ranks = np.array(sorted(rank.get(int(x), a.n) for x in day.anomaly_rows))
    # quiet vs active clients of the planted rows (dns / proxy): a client is "quiet" when it is in
    # the least active tenth of the day's clients by event count
    split = {}
    ccol = {"dns": "ip_dst", "proxy": "clientip"}.get(a.source)
    if ccol is not None and len(day.anomaly_rows):
        cli = np.asarray(day.cols[ccol])
        uc, inv, cnt = np.unique(cli, return_inverse=True, return_counts=True)
        quiet_max = np.sort(cnt)[max(0, uc.size // 10 - 1)]
        ar = np.asarray(day.anomaly_rows, dtype=np.int64)
        ev = cnt[inv[ar]]
        hit = np.array([rank.get(int(x), a.n) < a.maxresults for x in ar])
        q = ev <= quiet_max
        split = {"clients": int(uc.size), "quiet_client_max_events": int(quiet_max),
                 "planted_on_quiet_clients": int(q.sum()), "planted_on_active_clients": int((~q).sum()),
                 "recall_quiet": float(hit[q].mean()) if q.any() else None,
                 "recall_active": float(hit[~q].mean()) if (~q).any() else None,
                 "planted_client_events_p50": int(np.median(ev))}
    out = {"source": a.source, "n": a.n, "wide": a.wide, "kind": a.anomaly_kind, "K": K, "sweeps": a.sweeps,
           "lt_codebook": a.lt_codebook if a.source == "flow" and a.wide else None,
           "ms_per_sweep": round(res.timings.get("train_dev_s", res.timings.get("train_s", 0)) / a.sweeps * 1e3, 4),
           "vocab": int(res.lda.vocab.numel()), "anomalies": int(ranks.size),
           "recall_topN": float(np.mean(ranks < a.maxresults)), "maxresults": a.maxresults,
           "rank_p50": int(np.median(ranks)), "rank_max": int(ranks.max()), "ranks_head": ranks[:20].tolist(),
           "loglik": res.stats.get("loglik"), "wall_s": round(time.perf_counter() - t0, 1), **split}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
