#!/usr/bin/env python3
"""Equilibrium check of the samplers on a tiny planted corpus (60 docs, V = 80, K = 10, one chunk
per doc): mean collapsed log-likelihood over long chains of the slow exact textbook CGS
(spec.textbook_cgs), the dense sampler (AD-LDA word snapshot) and the MH sampler. Batch-means
standard errors.

  python tools/mh_equilibrium.py --burn 300 --sweeps 2000
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--burn", type=int, default=300)
    ap.add_argument("--sweeps", type=int, default=2000)
    a = ap.parse_args()
    import torch
    from scipy.special import gammaln

    from oni355.models.corpus import build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA, tiling_for
    from oni355.ref import spec
    r = np.random.default_rng(0)
    D, V, K = 60, 80, 10
    lens = r.integers(5, 90, D)
    phi = r.dirichlet(np.full(V, 0.05), K)
    th = r.dirichlet(np.full(K, 0.3), D)
    docs = []
    for d in range(D):
        z = r.choice(K, lens[d], p=th[d])
        docs.append(np.array([r.choice(V, p=phi[k]) for k in z]))
    tdoc = torch.from_numpy(np.repeat(np.arange(D), lens).astype(np.int32))
    tword = torch.from_numpy(np.concatenate(docs).astype(np.int32))
    alpha, beta, ev = 50 / K, 0.01, 2

    def ll_counts(ndk, nwk):
        nk, nd = nwk.sum(0), ndk.sum(1)
        return (K * (gammaln(V * beta) - V * gammaln(beta)) + gammaln(nwk + beta).sum() - gammaln(nk + V * beta).sum()
                + D * (gammaln(K * alpha) - K * gammaln(alpha)) + gammaln(ndk + alpha).sum()
                - gammaln(nd + K * alpha).sum())
    res = {}
    vals = []

    def cb(sw, z):
        if sw > a.burn and sw % ev == 0:
            ndk, nwk = np.zeros((D, K)), np.zeros((V, K))
            for d, (ws, zs) in enumerate(zip(docs, z)):
                np.add.at(ndk, (d, zs), 1)
                np.add.at(nwk, (ws, zs), 1)
            vals.append(ll_counts(ndk, nwk))
    spec.textbook_cgs(docs, V, K, alpha, beta, a.burn + a.sweeps, 1, on_sweep=cb)
    res["textbook"] = np.array(vals)
    for sampler in ("auto", "mh"):
        G, _ = tiling_for(K, sampler)
        c = build_corpus(tdoc, tword, D, V, torch.arange(D, dtype=torch.int32) * 3 + 1, G, L=96)
        m = GibbsLDA(c, GibbsConfig(K=K, sampler=sampler, post_samples=1, count_mode="recount"))
        m.initialize()
        m.sweep(a.burn)
        ll = []
        for _ in range(a.sweeps // ev):
            m.sweep(ev)
            ll.append(m.log_likelihood())
        res["dense" if sampler == "auto" else "mh"] = np.array(ll)
    out = {}
    for k, v in res.items():
        nb = 10
        b = v[: len(v) // nb * nb].reshape(nb, -1).mean(1)
        out[k] = {"mean_loglik": round(float(v.mean()), 1), "se": round(float(b.std(ddof=1) / np.sqrt(nb)), 1)}
    print(json.dumps({"burn": a.burn, "sweeps": a.sweeps, **out}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
