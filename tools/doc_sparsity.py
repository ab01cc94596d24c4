#!/usr/bin/env python3
"""How sparse are the K = 100 count tables a sweep samples against? (design input for a bucketed
sampler)

For each source's bench-size day trained for 200 sweeps at K = 100 it prints, token-weighted:
  * nnz(n_d·), the document's non-zero topics (what a doc-sparse bucket iterates over), both per
    token and per SELL wave step (a wave steps at the pace of its densest chunk);
  * nnz(n_·w), the word's non-zero topics (SparseLDA's word bucket);
  * the share of a token's weight Σ_k (n_dk + α) q_wk that is the α part α Σ_k q_wk (the share of
    draws a smoothing bucket answers without touching the document).

  python tools/doc_sparsity.py [flow|dns|proxy ...] [--n N] [--wide]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(x, w, qs=(0.5, 0.9, 0.99)):
    import numpy as np
    o = np.argsort(x)
    cw = np.cumsum(w[o]) / w.sum()
    return {f"p{int(q * 100)}": float(x[o][min(np.searchsorted(cw, q), x.size - 1)]) for q in qs}


def main() -> int:
    import numpy as np
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*", default=["flow", "dns", "proxy"])
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--wide", action="store_true")
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    for src in a.sources:
        n = a.n or (12_500_000 if src == "flow" else 2_000_000)
        kw = dict(K=a.K, sweeps=a.sweeps, maxresults=3000, device=dev)
        if src == "flow":
            from oni355.pipeline.flow import run_flow
            from oni355.synth.flow import generate_flows
            day = generate_flows(n, seed=7, n_hosts=max(64, n // 25), wide_vocab=a.wide)
            res = run_flow(day.cols, **kw)
        elif src == "dns":
            from oni355.pipeline.dns import run_dns
            from oni355.synth.dns import generate_dns
            day = generate_dns(n, seed=7, n_clients=max(32, n // 40), wide_vocab=0.5 if a.wide else 0.0)
            res = run_dns(day.cols, top_domains=day.top_domains, user_domain="intel", **kw)
        else:
            from oni355.pipeline.proxy import run_proxy
            from oni355.synth.proxy import generate_proxy
            day = generate_proxy(n, seed=7, n_clients=max(32, n // 40), wide_vocab=0.5 if a.wide else 0.0)
            res = run_proxy(day.cols, **kw)
        m = res.lda.model
        c = m.c
        K = a.K
        ndk = m.ndk_cur[: c.D, :K].long()
        nwk = m.nwk[:, :K].long()
        q = m.q[:, :K].double()
        tok_d = ndk.sum(1)
        nnz_d = (ndk > 0).sum(1)
        tok_w = nwk.sum(1)
        nnz_w = (nwk > 0).sum(1)
        # per pair: B = n_d · q_w, A = α Σ q_w (token-weighted by the pair count)
        pd, pw, pc = c.pair_doc.long(), c.pair_word.long(), c.pair_cnt.double()
        A = m.alpha * q.sum(1)[pw]
        B = torch.zeros_like(A)
        step = 1 << 20
        for i in range(0, pd.numel(), step):
            B[i:i + step] = (ndk[pd[i:i + step]].double() * q[pw[i:i + step]]).sum(1)
        share = (A / (A + B))
        # per SELL wave step: the densest chunk of the slice
        S = c.S
        cd = c.chunk_doc.long().view(-1, S)
        live = cd >= 0
        cn = torch.where(live, nnz_d[cd.clamp_min(0)], torch.zeros_like(cd))
        slice_max = cn.max(1).values.double()
        slice_tok = (torch.where(live, c.chunk_len.long().view(-1, S), torch.zeros_like(cd))).sum(1).double()
        slice_steps = c.slice_len.double()
        out = {
            "source": src, "n": n, "K": K, "T": int(c.T), "D": int(c.D), "V": int(c.V), "alpha": m.alpha,
            "nnz_doc_token_weighted": {"mean": float((nnz_d.double() * tok_d).sum() / tok_d.sum()),
                                       **pct(nnz_d.cpu().numpy(), tok_d.double().cpu().numpy())},
            "nnz_doc_wave_step_max": float((slice_max * slice_steps).sum() / slice_steps.sum()),
            "wave_lane_fill": float(slice_tok.sum() / (slice_steps.sum() * S)),
            "nnz_word_token_weighted": {"mean": float((nnz_w.double() * tok_w).sum() / tok_w.sum()),
                                        **pct(nnz_w.cpu().numpy(), tok_w.double().cpu().numpy())},
            "alpha_share_token_weighted": float((share * pc).sum() / pc.sum()),
            "alpha_share_p10_p50_p90": [float(x) for x in
                                        pct(share.cpu().numpy(), pc.cpu().numpy(), (0.1, 0.5, 0.9)).values()],
        }
        print(json.dumps(out), flush=True)
        del res, m
        if dev == "cuda":
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
