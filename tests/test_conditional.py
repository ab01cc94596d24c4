"""The sampler draws from the collapsed conditional with the token REMOVED from both sides
(SURVEY.md §2.6 K10 "remove its old z"; §4.3 sampler (d)).

* Exact-conditional check of the oracle the kernels replay bit for bit (oni355/ref/spec.py
  gibbs_pass, tested against k_gibbs_x1 / k_gibbs_ldsg / k_gibbs in test_gpu_kernels.py): every
  document is one token of the same word, starts from the same doc-topic row and from the same
  sweep-start snapshot -- which counts the token itself at its topic z0 -- so every chunk draws
  from p(k) ∝ (n_dk^¬t + α)(n_wk^¬t + β)/(n_k^¬t + Vβ) with its own Philox stream; the topic
  histogram must fit it (chi-square) for one-lane (G = 1) and multi-lane (G = 2, 4) units.
* Singleton words (the events the score ranks): a word seen once in the day has n_wk^¬t = 0 for
  every topic, so its token must NOT stay in its topic more often than the doc side says -- the
  snapshot's own count would otherwise give the old topic (1 + β)/β = 101× the word weight.
* Cross-check against the slow textbook sampler (spec.textbook_cgs): per-sweep stay rates of
  singleton-word and common-word tokens, from the same initial topics.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch
from scipy import stats

from oni355 import ops
from oni355.models.corpus import build_corpus, canonical_tokens
from oni355.models.gibbs import GibbsConfig, GibbsLDA
from oni355.ref import spec


def _state(K, D=40000, V=8, seed=3, singleton=False):
    G, KP = ops.choose_tiling(K)
    KS = G * KP
    r = np.random.default_rng(seed)
    c = build_corpus(torch.arange(D, dtype=torch.int32), torch.zeros(D, dtype=torch.int32), D, V,
                     torch.arange(D, dtype=torch.int32) * 7 + 1, G, L=64)
    nwk = np.zeros((V, KS), np.int32)
    hot = r.choice(K, size=max(K // 5, 3), replace=False)  # word 0: a sparse row (most topics empty)
    nwk[0, hot] = r.integers(1, 40, hot.size)
    if singleton:  # word 0 seen once: the token itself is its only count
        nwk[0] = 0
        nwk[0, hot[0]] = 1
    nwk[1:, :K] = r.integers(0, 30, (V - 1, K))
    nk = nwk.sum(0).astype(np.int32) + 5
    nk[K:] = 0
    row = np.zeros(KS, np.int32)
    row[:K] = r.integers(0, 6, K)
    z0 = int(hot[0])
    row[z0] += 1  # the token's own topic: removed before its draw (doc side and word side)
    tok_z = np.full(c.tok_word.numel(), 0, np.uint8)
    tok_z[c.tok_word.numpy() != np.int32(-1).view(np.int32)] = z0
    st = dict(tok_word=c.tok_word.numpy().view(np.uint32), tok_z=tok_z, slice_off=c.slice_off.numpy(),
              slice_len=c.slice_len.numpy(), chunk_doc=c.chunk_doc.numpy(), chunk_pos0=c.chunk_pos0.numpy(),
              chunk_key=c.chunk_key.numpy().view(np.uint32), chunk_multi=c.chunk_multi.numpy(),
              ndk_src=np.tile(row, (D, 1)), ndk_dst=np.zeros((D, KS), np.int32),
              dnwk=np.zeros((V, KS), np.int32), dnk=np.zeros(KS, np.int32))
    return c, st, nwk, nk, row, z0, G, KP


def _draw(K, alpha, beta, singleton=False):
    c, st, nwk, nk, row, z0, G, KP = _state(K, singleton=singleton)
    V = nwk.shape[0]
    vbeta = float(np.float32(V * beta))
    _, _, q, qfix = spec.gibbs_apply(nwk, np.zeros_like(nwk), np.zeros_like(nk), nk, K, beta, vbeta)
    st["q"], st["qfix"] = q, qfix
    s0, s1 = spec.split_seed(12345)
    spec.gibbs_pass(st, G, KP, K, alpha, s0, s1, False, 1, c.chunk_len.numpy())
    live = st["tok_word"] != np.uint32(0xFFFFFFFF)
    z = st["tok_z"][live].astype(np.int64)
    # the collapsed conditional, token removed from the doc row, the word row and the topic total
    n = row[:K].astype(np.float64)
    nw = nwk[0, :K].astype(np.float64)
    nt = nk[:K].astype(np.float64)
    n[z0] -= 1
    nw[z0] -= 1
    nt[z0] -= 1
    p = (n + alpha) * (nw + beta) / (nt + V * beta)
    return z, p / p.sum(), z0


def _chi2(z, p, K):
    obs = np.bincount(z, minlength=K)[:K]
    exp = p * obs.sum()
    rare = exp < 5  # pool the rare topics into one cell so every expected count is >= 5
    o = np.append(obs[~rare], obs[rare].sum())
    e = np.append(exp[~rare], exp[rare].sum())
    if e[-1] == 0:
        o, e = o[:-1], e[:-1]
    return stats.chisquare(o, e)


@pytest.mark.parametrize("K", [20, 7, 32, 40, 50, 100])
def test_draws_follow_the_collapsed_conditional(K):
    z, p, _ = _draw(K, 0.3, 0.05)
    assert z.size == 40000
    chi2, pv = _chi2(z, p, K)
    assert pv > 1e-4, (chi2, pv)


@pytest.mark.parametrize("K", [20, 50])
def test_singleton_word_token_is_not_pinned_to_its_topic(K):
    alpha, beta = 2.5, 0.01
    z, p, z0 = _draw(K, alpha, beta, singleton=True)
    chi2, pv = _chi2(z, p, K)
    assert pv > 1e-4, (chi2, pv)
    # the stay probability is the doc side's alone: nothing like the 101x word weight of z0
    stay = float((z == z0).mean())
    assert abs(stay - p[z0]) < 0.01, (stay, p[z0])
    assert stay < 0.2, stay


def _verdict_corpus(seed=11, D=400, K=20):
    """400 docs of 20-119 tokens over a Zipf vocabulary, 5 % of tokens on day-unique words."""
    r = np.random.default_rng(seed)
    lens = r.integers(20, 120, D)
    tdoc = np.repeat(np.arange(D), lens)
    T = tdoc.size
    V0 = 600
    tword = (r.zipf(1.4, T) - 1) % V0
    uniq = r.random(T) < 0.05
    tword[uniq] = V0 + np.arange(int(uniq.sum()))
    V = V0 + int(uniq.sum())
    o = np.lexsort((tword, tdoc))
    return tdoc[o], tword[o], D, V


def test_stay_rates_match_textbook_collapsed_gibbs():
    tdoc, tword, D, V = _verdict_corpus()
    K, alpha, beta = 20, 2.5, 0.01
    keys = torch.arange(D, dtype=torch.int32) * 13 + 5
    c = build_corpus(torch.from_numpy(tdoc), torch.from_numpy(tword), D, V, keys, 1, L=128)
    m = GibbsLDA(c, GibbsConfig(K=K, alpha=alpha, beta=beta, seed=9, count_mode="atomic", post_samples=1,
                                sampler="dense"))
    m.initialize()
    cdoc, cword = (t.numpy() for t in canonical_tokens(c))
    wc = np.bincount(cword, minlength=V)
    single = wc[cword] == 1
    common = wc[cword] >= 50
    assert single.sum() > 1000 and common.sum() > 5000
    sweeps = 5
    prod = {"s": [], "c": []}
    z = m.canonical_z().numpy().astype(np.int64)
    z0 = z.copy()
    for _ in range(sweeps):
        m.sweep(1)
        zn = m.canonical_z().numpy().astype(np.int64)
        prod["s"].append(float((zn == z)[single].mean()))
        prod["c"].append(float((zn == z)[common].mean()))
        z = zn
    # textbook CGS from the same initial topics (documents in canonical token order)
    starts = np.concatenate([[0], np.cumsum(np.bincount(cdoc, minlength=D))])
    docs = [cword[starts[d]:starts[d + 1]] for d in range(D)]
    zdocs = [z0[starts[d]:starts[d + 1]] for d in range(D)]
    tb = {"s": [], "c": []}
    prev = [np.array(a) for a in zdocs]

    def on_sweep(_, zz):
        cur = np.concatenate(zz)
        before = np.concatenate(prev)
        tb["s"].append(float((cur == before)[single].mean()))
        tb["c"].append(float((cur == before)[common].mean()))
        for i, a in enumerate(zz):
            prev[i] = a.copy()

    spec.textbook_cgs(docs, V, K, alpha, beta, sweeps, seed=4, z0=zdocs, on_sweep=on_sweep)
    for s in range(sweeps):
        assert abs(prod["s"][s] - tb["s"][s]) < 0.03, (s, prod, tb)
        assert abs(prod["c"][s] - tb["c"][s]) < 0.03, (s, prod, tb)
    # and far from the old bias (0.8+ stay rate for singleton tokens)
    assert max(prod["s"]) < 0.2, prod
