#!/usr/bin/env python3
"""Oracle recall next to LDA recall (VERDICT r5 "next round" item 2).

For each case: generate the synthetic day, run the product's pipeline (the same run_flow /
run_dns / run_proxy as oni-ml) and rank the planted rows; then score every event with the label
oracle (oni355.synth.oracle: the generators' own labels, counts over the normal rows only) and
report both recalls at the top-3000 / 15000 / 45000.

  python tools/oracle_recall.py --case flow-realistic-12.5M [--case ...] --out gpurun_out/oracle.jsonl

Cases (name → source, events, vocabulary, K, anomaly kind): see CASES.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TOPS = (3000, 15000, 45000)
# name: (source, events, realistic vocabulary, K, anomaly kind, flow shards)
CASES = {
    "flow-default-12.5M": ("flow", 12_500_000, False, 20, None, 1),
    "flow-realistic-12.5M": ("flow", 12_500_000, True, 20, None, 1),
    "flow-config5-share": ("flow", 62_500_000, True, 100, None, 4),
    "dns-config5-share": ("dns", 31_250_000, True, 100, None, 1),
    "proxy-config5-share": ("proxy", 31_250_000, True, 100, None, 1),
    "dns-realistic-own-client-2M": ("dns", 2_000_000, True, 50, "rare-active", 1),
    "proxy-realistic-own-client-2M": ("proxy", 2_000_000, True, 20, "rare-active", 1),
    "dns-realistic-quiet-2M": ("dns", 2_000_000, True, 50, "rare", 1),
    "proxy-realistic-quiet-2M": ("proxy", 2_000_000, True, 20, "rare", 1),
    # small CPU-sized cases (tests / smoke)
    "flow-realistic-200k": ("flow", 200_000, True, 20, None, 1),
    "dns-realistic-own-client-100k": ("dns", 100_000, True, 50, "rare-active", 1),
}


def _day(src, n, wide, kind, shards, seed):
    if src == "flow":
        from oni355.synth.flow import generate_flows, generate_flows_sharded
        if shards > 1:
            return generate_flows_sharded(n // shards, shards, seed=seed, n_hosts=max(64, n // 25), procs=8,
                                          wide_vocab=wide)
        return generate_flows(n, seed=seed, n_hosts=max(64, n // 25), wide_vocab=wide)
    kw = {"anomaly_kind": kind} if kind else {}
    if src == "dns":
        from oni355.synth.dns import generate_dns
        return generate_dns(n, seed=seed, n_clients=max(32, n // 40), wide_vocab=0.5 if wide else 0.0, **kw)
    from oni355.synth.proxy import generate_proxy
    return generate_proxy(n, seed=seed, n_clients=max(32, n // 40), wide_vocab=0.5 if wide else 0.0, **kw)


def _tokens(src, day, device):
    """(doc keys per token slot, word keys per token slot) of every event, from the product's own
    featurizers (the words the LDA model sees)."""
    import torch
    if src == "flow":
        from oni355.pipeline import flow as pf
        d = pf.to_device(day.cols, device)
        cuts = pf.compute_cuts(d, None)
        sw, dw = pf.wordify(d, cuts)
        return ([d["sip"].to(torch.int64), d["dip"].to(torch.int64)],
                [sw.to(torch.int64) & 0xFFFFFFFF, dw.to(torch.int64) & 0xFFFFFFFF])
    if src == "dns":
        from oni355.pipeline import dns as pd
        d = pd.to_device(day.cols, device)
        words, _, _ = pd.featurize(d, None, pd.top_set(day.top_domains), "intel")
        return [d["ip_dst"].to(torch.int64)], [words.to(torch.int64)]
    from oni355.pipeline import proxy as pp
    from oni355.pipeline.dns import top_set
    from oni355.synth.dns import top_domain_list
    words, _, _ = pp.featurize(day.cols, device, None, top_set(top_domain_list()))
    docs = torch.from_numpy(np.asarray(day.cols["clientip"], np.uint32).astype(np.int64))
    return [docs], [words.to(torch.int64)]


def _anatomy(day, rows, planted, docs, words, orc, src, top=3000):
    """What fills the LDA top-N: label kind of each row (planted / behaviour profile / long-tail
    behaviour), how often its rarest word occurs among the day's tokens, its documents' sizes;
    and where the missed planted rows and the top-N normal rows sit in the smoothed oracle."""
    import torch
    lab = np.asarray(day.labels)
    P = 20 if src == "flow" else None
    n = lab.size
    wk = torch.cat([w.reshape(-1).cpu() for w in words])
    dk = torch.cat([d.reshape(-1).cpu() for d in docs])
    _, winv, wcnt = torch.unique(wk, return_inverse=True, return_counts=True)
    _, dinv, dcnt = torch.unique(dk, return_inverse=True, return_counts=True)
    S = len(words)
    wc = wcnt[winv].view(S, n).min(0).values.numpy()   # the event's rarest word's day count
    dc = dcnt[dinv].view(S, n).min(0).values.numpy()   # its smaller document
    head = rows[:top]
    normal = head[lab[head] >= 0]
    kinds = {"planted": int((lab[head] < 0).sum())}
    if P is not None:
        kinds["profile"] = int(((lab[normal] >= 0) & (lab[normal] < P)).sum())
        kinds["long_tail"] = int((lab[normal] >= P).sum())
    sm = orc["loo_smooth"]
    order = np.argsort(sm, kind="stable")
    srank = np.empty(n, np.int64)
    srank[order] = np.arange(n)
    missed = planted[~np.isin(planted, head)]
    q = lambda a: [int(x) for x in np.percentile(a, [10, 50, 90])] if len(a) else None  # noqa: E731
    return {"top": top, "kinds": kinds,
            "normal_top_word_count_p10_50_90": q(wc[normal]), "normal_top_doc_tokens_p10_50_90": q(dc[normal]),
            "normal_top_singleton_words": int((wc[normal] == 1).sum()),
            "normal_top_smooth_oracle_rank_p10_50_90": q(srank[normal]),
            "missed_planted": int(missed.size), "missed_word_count_p10_50_90": q(wc[missed]),
            "missed_doc_tokens_p10_50_90": q(dc[missed]), "missed_lda_rank_p10_50_90":
            q(np.array([int(np.nonzero(rows == m)[0][0]) if (rows == m).any() else len(rows) for m in missed])),
            "planted_word_count_p10_50_90": q(wc[planted]), "planted_doc_tokens_p10_50_90": q(dc[planted])}


def run_case(name, device, sweeps, seed, K=None, beta=None, alpha=None, anatomy=False):
    import torch
    from oni355.synth.oracle import expected_recall, label_oracle
    src, n, wide, K0, kind, shards = CASES[name]
    K = K or K0
    t0 = time.perf_counter()
    day = _day(src, n, wide, kind, shards, seed)
    gen_s = time.perf_counter() - t0
    kw = dict(K=K, sweeps=sweeps, maxresults=max(TOPS), device=device)
    if beta is not None:
        kw["beta"] = beta
    if alpha is not None:
        kw["alpha"] = alpha
    if src == "flow":
        from oni355.pipeline.flow import run_flow
        res = run_flow(day.cols, **kw)
    elif src == "dns":
        from oni355.pipeline.dns import run_dns
        res = run_dns(day.cols, top_domains=day.top_domains, user_domain="intel", **kw)
    else:
        from oni355.pipeline.proxy import run_proxy
        from oni355.synth.dns import top_domain_list
        res = run_proxy(day.cols, top_domains=top_domain_list(), **kw)
    planted = np.asarray(day.anomaly_rows, dtype=np.int64)
    rows = np.asarray(res.rows, dtype=np.int64)
    lda = {str(t): round(float(np.isin(planted, rows[:t]).mean()), 4) for t in TOPS}
    vocab = int(res.lda.vocab.numel())
    del res
    if device != "cpu":
        torch.cuda.empty_cache()
    docs, words = _tokens(src, day, device)
    orc = label_oracle(docs, words, day.labels, device=device)
    out = {"case": name, "source": src, "events": n, "realistic_vocab": wide, "K": K, "sweeps": sweeps,
           "alpha": alpha, "beta": beta, "anomaly_kind": kind or "default", "planted": int(planted.size),
           "vocab": vocab, "lda_recall": lda}
    if anatomy:
        out["anatomy"] = _anatomy(day, rows, planted, docs, words, orc, src)
    for k in ("leave_in", "loo", "loo_smooth"):
        out[f"oracle_{k}_recall"] = {str(t): round(expected_recall(orc[k], planted, t), 4) for t in TOPS}
    # anatomy: planted rows whose (every) word no normal row of the day carries (oracle score 0)
    out["planted_oracle_zero"] = int((orc["leave_in"][planted] == 0).sum())
    out["normal_rows_loo_zero"] = int((orc["loo"] == 0).sum()) - int((orc["loo"][planted] == 0).sum())
    out["wall_s"] = round(time.perf_counter() - t0, 1)
    out["gen_s"] = round(gen_s, 1)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", action="append", required=True, choices=sorted(CASES))
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--out", default=None)
    ap.add_argument("--topics", type=int, default=None, help="estimator A/B: K instead of the case's")
    ap.add_argument("--beta", type=float, default=None, help="estimator A/B: β")
    ap.add_argument("--alpha", type=float, default=None, help="estimator A/B: α (default 50/K)")
    ap.add_argument("--anatomy", action="store_true", help="describe the LDA top-N rows (label kind, word counts)")
    a = ap.parse_args()
    for name in a.case:
        r = run_case(name, a.device, a.sweeps, a.seed, K=a.topics, beta=a.beta, alpha=a.alpha, anatomy=a.anatomy)
        line = json.dumps(r)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
