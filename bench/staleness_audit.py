#!/usr/bin/env python3
"""Doc-side staleness audit: does the chunk length L change
what 200 sweeps converge to?

Every chunk of a document longer than L samples against the sweep-start n_dk row of its document
(the same AD-LDA staleness the word side has), so most tokens of a heavy IP see a doc state one
sweep old. This runs the same day at several L -- down to one chunk per document (an exact
sequential chain on the doc side) -- and records, per configuration: the collapsed log-likelihood
every ``--every`` sweeps, the ms per sweep, planted-anomaly recall in the top-N and the overlap of
its top-N with the exact chain's (or the largest L's).

  python bench/staleness_audit.py --flows 1000000 --chunk-lens 128,128@1,1024,4096,0
      # 0 = one chunk per doc; L@s = chunk length L with the LDA seed offset by s (the top-N overlap
      # of two seeds at the same L is the yardstick for the overlap across L)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--chunk-lens", default="128,1024,4096,0")
    ap.add_argument("--maxresults", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    import numpy as np
    import torch

    from oni355.pipeline import common, flow
    from oni355.synth.flow import generate_flows

    dev = torch.device(a.device)
    day = generate_flows(a.flows, seed=a.seed, n_hosts=max(64, a.flows // 25))
    d = flow.to_device(day.cols, dev)
    cuts = flow.compute_cuts(d, None)
    sw, dw = flow.wordify(d, cuts)
    n = d["sip"].numel()
    dk = torch.cat([common.u32_to_i64(d["sip"]), common.u32_to_i64(d["dip"])])
    wk = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
    vocab, wids = common.encode_words(wk.contiguous(), None, key_bits=32)
    _, inv = torch.unique(dk, return_inverse=True)
    max_len = int(torch.bincount(inv).max())
    results = {}
    for spec_ in a.chunk_lens.split(","):
        L, _, so = spec_.partition("@")
        L, so = int(L), int(so or 0)
        Lr = max_len if L == 0 else L
        t0 = time.perf_counter()
        run = common.build_and_train(dk, None, None, vocab, a.topics, None, 0.01, 0x0D15EA5E + so, 0, Lr, None,
                                     word_ids=wids, n_event0=n, train=False)
        m = run.model
        m.initialize()
        trace, ms = [], []
        done = 0
        while done < a.sweeps:
            k = min(a.every, a.sweeps - done)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t1 = time.perf_counter()
            m.sweep(k)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            ms.append((time.perf_counter() - t1) / k * 1e3)
            done += k
            trace.append((done, m.log_likelihood()))
        theta, phi = m.theta(), m.phi()
        if run.pairs is not None:
            plan = common.plan_from_pairs(run.pairs, n, 2)
        else:
            plan = common.event_score_plan(run, run.doc_keys64, vocab, [dk[:n], dk[n:]], wids, [wk[:n], wk[n:]], None)
        hist = torch.zeros(2048, dtype=torch.int32, device=dev)
        score, _, _ = common.plan_score(theta, phi, plan, 1.0, hist=hist)
        rows, _ = common.top_n(score, 1.0, a.maxresults, None, hist=hist, order=plan.order)[:2]
        rows = rows.cpu().numpy()
        c = run.corpus
        key = spec_
        results[key] = {"chunk_len": Lr, "seed_offset": so, "one_chunk_per_doc": L == 0,
                        "long_docs": int(c.long_rows.numel()),
                        "slices": c.n_slices, "loglik_trace": trace, "ms_per_sweep_median": float(np.median(ms)),
                        "recall_topN": float(np.isin(day.anomaly_rows, rows).mean()), "rows": rows,
                        "wall_s": round(time.perf_counter() - t0, 2)}
        print(json.dumps({k: v for k, v in results[key].items() if k != "rows"}), flush=True)
        del run, m
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    ref = results.get("0") or max(results.values(), key=lambda r: r["chunk_len"])
    summary = {"flows": a.flows, "max_doc_len": max_len, "reference": "one chunk per doc" if "0" in results else
               f"L={ref['chunk_len']}", "configs": []}
    for key, r in results.items():
        summary["configs"].append({"config": key, "chunk_len": r["chunk_len"], "seed_offset": r["seed_offset"],
                                   "final_loglik": r["loglik_trace"][-1][1],
                                   "loglik_at_100": dict(r["loglik_trace"]).get(100),
                                   "recall_topN": r["recall_topN"], "ms_per_sweep": round(r["ms_per_sweep_median"], 4),
                                   "topN_overlap_with_reference": float(np.isin(r["rows"], ref["rows"]).mean())})
    print(json.dumps(summary), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
