"""Exact-conditional check of the word-sparse samplers' numerics (oni355/ref/spec.py gibbs_pass_ws /
gibbs_pass_wsg -- the specifications k_gibbs_ws / k_gibbs_wsg are tested bitwise against in
test_gpu_kernels.py). Every document of the corpus is one token of the same word and starts from
the same doc-topic row, so every chunk draws from the same collapsed conditional
p(k) ∝ (n_dk^-t + α)(n_wk + β)/(n_k + Vβ) with its own Philox stream: the topic histogram over the
chunks must fit that distribution (chi-square), for the one-lane and the G-lane decomposition
(word bucket + smoothing bucket, lanes combined by the scan) alike, and for the dense oracle."""
from __future__ import annotations

import numpy as np
import pytest
import torch
from scipy import stats

from oni355 import ops
from oni355.models.corpus import build_corpus
from oni355.ref import spec


def _state(K, D=40000, V=8, seed=3):
    G, KP = ops.choose_tiling(K)
    KS = G * KP
    r = np.random.default_rng(seed)
    c = build_corpus(torch.arange(D, dtype=torch.int32), torch.zeros(D, dtype=torch.int32), D, V,
                     torch.arange(D, dtype=torch.int32) * 7 + 1, G, L=64)
    nwk = np.zeros((V, KS), np.int32)
    hot = r.choice(K, size=max(K // 5, 3), replace=False)  # word 0: a sparse row (most topics empty)
    nwk[0, hot] = r.integers(1, 40, hot.size)
    nwk[1:, :K] = r.integers(0, 30, (V - 1, K))
    nk = nwk.sum(0).astype(np.int32) + 5
    nk[K:] = 0
    row = np.zeros(KS, np.int32)
    row[:K] = r.integers(0, 6, K)
    z0 = int(hot[0])
    row[z0] += 1  # the token's own topic: removed before its draw
    tok_z = np.full(c.tok_word.numel(), 0, np.uint8)
    tok_z[c.tok_word.numpy() != np.int32(-1).view(np.int32)] = z0
    st = dict(tok_word=c.tok_word.numpy().view(np.uint32), tok_z=tok_z, slice_off=c.slice_off.numpy(),
              slice_len=c.slice_len.numpy(), chunk_doc=c.chunk_doc.numpy(), chunk_pos0=c.chunk_pos0.numpy(),
              chunk_key=c.chunk_key.numpy().view(np.uint32), chunk_multi=c.chunk_multi.numpy(),
              ndk_src=np.tile(row, (D, 1)), ndk_dst=np.zeros((D, KS), np.int32),
              dnwk=np.zeros((V, KS), np.int32), dnk=np.zeros(KS, np.int32))
    return c, st, nwk, nk, row, z0, G, KP


@pytest.mark.parametrize("K,sampler", [(20, "dense"), (20, "ws"), (40, "ws"), (40, "wsg"), (100, "wsg"),
                                       (64, "wsg")])
def test_word_sparse_draws_follow_the_collapsed_conditional(K, sampler):
    alpha, beta = 0.3, 0.05
    c, st, nwk, nk, row, z0, G, KP = _state(K)
    V = nwk.shape[0]
    vbeta = V * beta
    s0, s1 = spec.split_seed(12345)
    cl = c.chunk_len.numpy()
    if sampler == "dense":
        st["q"] = ((nwk.astype(np.float32) + np.float32(beta)) / (nk.astype(np.float32) + np.float32(vbeta)))
        st["q"][:, K:] = 0
        spec.gibbs_pass(st, G, KP, K, alpha, s0, s1, False, 1, cl, fma=True)
    else:
        tabs = spec.ws_tables(nwk, nk, K, beta, vbeta)
        if sampler == "ws":
            spec.gibbs_pass_ws(st, G, K, alpha, s0, s1, 1, cl, tabs)
        else:
            spec.gibbs_pass_wsg(st, G, KP, K, alpha, s0, s1, 1, cl, tabs)
    live = st["tok_word"] != np.uint32(0xFFFFFFFF)
    z = st["tok_z"][live].astype(np.int64)
    n = row[:K].astype(np.float64)
    n[z0] -= 1
    p = (n + alpha) * (nwk[0, :K] + beta) / (nk[:K] + vbeta)
    p /= p.sum()
    obs = np.bincount(z, minlength=K)[:K]
    assert obs.sum() == live.sum() == 40000
    exp = p * obs.sum()
    # pool the rare topics into one cell so every expected count is >= 5
    rare = exp < 5
    o = np.append(obs[~rare], obs[rare].sum())
    e = np.append(exp[~rare], exp[rare].sum())
    if e[-1] == 0:
        o, e = o[:-1], e[:-1]
    chi2, pv = stats.chisquare(o, e)
    assert pv > 1e-4, (chi2, pv, obs, np.round(exp, 1))
