"""The Metropolis-Hastings sampler (spec.gibbs_pass_mh / k_gibbs_mh) leaves the collapsed
conditional invariant (verdict r3 next-round item 2: "exact-stationary under MH").

Stationarity check of the oracle's token moves (spec.mh_moves): for a token with fixed other
counts, π(k) ∝ (n_dk^¬ + α)·q'_k does not depend on the token's own topic zo. Each replica draws zo
from π, builds the sweep-start state that CONTAINS the token at zo (doc row b, q row with q_zo such
that fma(q_zo, A_zo, −B_zo) = q'_zo, the word's level-1 CDF of that q row) and runs the MH moves
from zo with its own Philox stream. If every move is a correct MH step, the output topics are again
distributed as π (chi-square), for one-chunk documents (proposals from the chunk's other tokens)
and documents over several chunks (proposals from the sweep-start row's alias table), one and two
cycles. Plus: the alias tables and the two-level word CDF reproduce their weights, and the MH chain
runs through GibbsLDA.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch
from scipy import stats

from oni355.ref import spec

F32 = np.float32


def _case(K, alpha, multi, R=120_000, Ld=7, s=2, seed=5, beta=0.01, V=50, stale=True):
    """R replicas of one token whose rest (every other count) is fixed; the sweep-start state of
    replica i holds the token at zo_i ~ π."""
    r = np.random.default_rng(seed)
    nn = np.zeros(K, np.int64)
    others = r.integers(0, K, Ld - 1)
    others[: Ld // 2] = others[0]  # a peaked doc side
    np.add.at(nn, others, 1)
    if multi and stale:
        nn += r.integers(0, 9, K) * (r.random(K) < 0.4)  # other chunks' tokens
    nw_rest = (r.integers(0, 4, K) * (r.random(K) < 0.5)).astype(np.int64)  # a rare word
    nk_rest = nw_rest + r.integers(5, 400, K)
    vbeta = F32(V * beta)
    qrest = (nw_rest + beta) / (nk_rest + float(vbeta))
    pi = (nn + alpha) * qrest
    pi /= pi.sum()
    zo = r.choice(K, size=R, p=pi)
    # snapshot with the token at z (k_apply's numerics): q rows, qfix, g and the word's proposal
    # tables (alias row + sum, CDF row)
    qrows, qfixes, gs, wcd, wal, wsums = [], [], [], [], [], []
    for z in range(K):
        nw = nw_rest.copy(); nw[z] += 1
        nk = nk_rest.copy(); nk[z] += 1
        den = nk.astype(F32) + vbeta
        q = ((nw.astype(F32) + F32(beta)) / den).astype(F32)
        qrows.append(q)
        qfixes.append(spec.gibbs_qfix(nk.astype(np.int32), K, float(vbeta)))
        wcd.append(spec.word_cdf(q[None, :], K)[0])
        t, tot = spec.alias_table(q[None, :])
        wal.append(t[0]); wsums.append(tot[0])
        gs.append((F32(1) / (den + F32(1))).astype(F32))
    qrows, wcd, gs, wal, wsums = map(np.array, (qrows, wcd, gs, wal, wsums))
    qrow = qrows[zo]
    qe = np.array([spec.excluded_q(qrows[z][z:z + 1], np.array([z]), qfixes[z])[0] for z in range(K)])[zo]
    # sweep-start doc row: the chunk's view without the token + stale counts of other chunks + the token
    bb = np.tile(nn, (R, 1)).astype(np.int32)
    if multi and stale:
        bb += r.integers(0, 3, (R, K)).astype(np.int32)
    bb[np.arange(R), zo] += 1
    drows = spec.alias_table((bb.astype(F32) + F32(alpha)).astype(F32))[0] if multi else None
    zslice = np.tile(np.insert(others, s, 0), (R, 1)).astype(np.int64)
    zslice[:, s] = zo
    return pi, zo, dict(nn=np.tile(nn, (R, 1)).astype(np.int32), bb=bb, qrow=qrow, zo=zo, qe=qe,
                        multi=np.full(R, multi), Nd=np.full(R, Ld - 1), s=s, zslice=zslice, drows=drows,
                        wcdf=wcd[zo], wrows=wal[zo], wsum=wsums[zo], gs=gs)


@pytest.mark.parametrize("K,alpha", [(7, 0.5), (20, 2.5), (9, 50 / 9)])
@pytest.mark.parametrize("multi", [False, True, "sparse"])
@pytest.mark.parametrize("doc_moves", [1, 2, 4])
@pytest.mark.parametrize("word", ["alias", "cdf"])
def test_mh_moves_leave_the_conditional_invariant(K, alpha, multi, doc_moves, word):
    # "sparse": a multi-chunk doc whose sweep-start row holds just its chunk (b_zo = 1 is common, so
    # the table's copy of the token at zo matters most)
    pi, zo, a = _case(K, alpha, bool(multi), stale=multi != "sparse")
    R = zo.size
    pos = np.arange(R, dtype=np.uint32)
    key = (np.arange(R, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
    zn = np.empty(R, np.int64)
    # g_t = 1/(D_t + 1) of the snapshot at t ≠ zo does not depend on zo: take it from any other z
    for z in range(K):
        m = zo == z
        if not m.any():
            continue
        g = a["gs"][(z + 1) % K].copy()
        sub = {k: (v[m] if isinstance(v, np.ndarray) and v.shape[:1] == (R,) else v) for k, v in a.items()}
        zn[m] = spec.mh_moves(sub["nn"], sub["bb"], sub["qrow"], sub["zo"], sub["qe"], sub["multi"], sub["Nd"],
                              a["s"], sub["zslice"], sub["drows"], sub["wcdf"] if word == "cdf" else sub["wrows"],
                              None if word == "cdf" else sub["wsum"], g, pos[m], key[m], 11,
                              0x1234, 0x5678, K, alpha, doc_moves)
    moved = float((zn != zo).mean())
    assert moved > 0.05, moved  # the moves are not all rejected
    obs = np.bincount(zn, minlength=K)
    exp = pi * R
    keep = exp >= 5
    chi = stats.chisquare(obs[keep], exp[keep] * obs[keep].sum() / exp[keep].sum())
    assert chi.pvalue > 1e-4, (chi, obs, np.round(exp))


def test_alias_tables_reproduce_their_weights():
    r = np.random.default_rng(1)
    for K in (3, 20, 100, 255):
        w = (r.random((64, K)) ** 4 + 1e-4).astype(F32)
        t, tot = spec.alias_table(w)
        assert np.allclose(tot, w.sum(1), rtol=1e-5)
        thr = (t >> 8).astype(np.int64)
        al = (t & 0xFF).astype(np.int64)
        P = np.zeros((64, K))
        rows = np.arange(64)
        for j in range(K):
            pr = thr[:, j] / 2.0 ** 24
            P[rows, j] += pr / K
            np.add.at(P, (rows, al[:, j]), (1 - pr) / K)
        ref = w / w.sum(1, keepdims=True, dtype=np.float64)
        assert np.abs(P - ref).max() < 2e-6
        # a draw uses the same tables
        rr = r.integers(0, 1 << 32, 200_000, dtype=np.uint64).astype(np.uint32)
        got = spec.alias_draw(np.repeat(t[:1], rr.size, 0), rr, K)
        h = np.bincount(got, minlength=K) / rr.size
        assert np.abs(h - ref[0]).max() < 0.01


@pytest.mark.parametrize("K", [3, 7, 20, 100, 129, 255])
def test_word_cdf_draw_reproduces_q(K):
    """The two-level inverse CDF draws topic k with probability q_k / Σq (buckets of 8 topics up to
    K = 128, 16 above; padding and empty topics never drawn)."""
    r = np.random.default_rng(K)
    q = (r.random((1, K)) ** 5 * 0.2).astype(F32)
    q[0, r.integers(0, K, max(1, K // 5))] = 0  # empty topics
    C = spec.word_cdf(q, K)
    assert np.isclose(C[0, -1], q.sum(), rtol=1e-5)
    n = 400_000
    rr = r.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    got = spec.word_cdf_draw(np.repeat(C, n, 0), np.repeat(q, n, 0), rr, K)
    h = np.bincount(got, minlength=K) / n
    ref = q[0] / q[0].sum(dtype=np.float64)
    assert got.max() < K and not h[ref == 0].any()
    assert np.abs(h - ref).max() < 0.006, np.abs(h - ref).max()


def test_mh_chain_through_the_model_cpu():
    from oni355.models.corpus import build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA, tiling_for
    r = np.random.default_rng(0)
    D, V, K = 300, 60, 40
    lens = r.integers(1, 200, D)  # short docs (one chunk) and long ones (several)
    tdoc = torch.from_numpy(np.repeat(np.arange(D), lens).astype(np.int32))
    tword = torch.from_numpy((r.zipf(1.5, tdoc.numel()) % V).astype(np.int32))
    G, _ = tiling_for(K, "mh")
    assert G == 1
    c = build_corpus(tdoc, tword, D, V, torch.arange(D, dtype=torch.int32) * 3 + 1, G, L=64)
    m = GibbsLDA(c, GibbsConfig(K=K, sampler="mh", count_mode="auto", post_samples=1, check_invariants=True))
    m.initialize()
    ll0 = m.log_likelihood()
    m.sweep(12)
    m.check_invariants()
    assert m.log_likelihood() > ll0
    with pytest.raises(ValueError):
        GibbsLDA(build_corpus(tdoc, tword, D, V, torch.arange(D, dtype=torch.int32) * 3 + 1, G, L=128),
                 GibbsConfig(K=K, sampler="mh"))
