"""Posterior-average sums at config-4/5 count magnitudes.

S = 50 samples of an int32 count wrap an int32 sum once the count passes 2^31 / S ≈ 42.9M -- one
topic's share of a 200M-token (config 4) or 1B-token (config 5) corpus. The sums are int64
(GibbsLDA.plan_average), added inside k_apply in contiguous windows (ops.gibbs_apply ``acc``),
and k_theta_rows / k_phi_rows read them wide. Planted counts just above that threshold must give
θ/φ equal to a float64 reference; a model whose token count could wrap an int32 table is refused.
"""
import numpy as np
import pytest
import torch

from oni355 import ops
from oni355.models import gibbs as gm
from oni355.models.corpus import build_corpus
from oni355.models.gibbs import GibbsConfig, GibbsLDA
from oni355.utils.checkpoint import Checkpointer

S = 50
BIG = 2**31 // S + 1_234_567  # S of these wrap an int32 sum


def _model(dev, K=20, sweeps=200, **cfg):
    r = np.random.default_rng(3)
    D, V = 40, 30
    lens = r.integers(5, 60, D)
    tdoc = np.repeat(np.arange(D), lens)
    tword = r.integers(0, V, tdoc.size)
    o = np.lexsort((tword, tdoc))
    keys = torch.arange(D, dtype=torch.int32) * 7 + 1
    c = build_corpus(torch.from_numpy(tdoc[o]).to(dev), torch.from_numpy(tword[o]).to(dev), D, V, keys.to(dev),
                     gm.tiling_for(K, "dense")[0], L=64)
    m = GibbsLDA(c, GibbsConfig(K=K, seed=5, sampler="dense", **cfg))
    m.initialize()
    m.plan_average(sweeps)
    return m


def _plant(m):
    """Counts just above 2^31 / S in n_wk, n_k and n_dk (+ small per-cell variation)."""
    K = m.K
    g = torch.Generator().manual_seed(1)
    wk = (BIG + torch.randint(0, 1000, (m.V, K), generator=g)).to(torch.int32)
    dk = (BIG + torch.randint(0, 1000, (m.ndk[0].shape[0], K), generator=g)).to(torch.int32)
    nk = (BIG + torch.randint(0, 1000, (K,), generator=g)).to(torch.int32)
    return wk, nk, dk


def _reference(m, wk, nk, dk):
    """θ, φ of S identical samples in float64."""
    K, a, b = m.K, m.alpha, m.beta
    wk, nk, dk = (t.to(torch.float64) * S for t in (wk, nk, dk))
    th = (dk + S * a) / (dk.sum(1, keepdim=True) + S * K * a)
    ph = (wk + S * b) / (nk + S * np.float32(m.vbeta))
    return th, ph


def _plant_tables(m, wk, nk, dk):
    """Put the planted counts in the model's tables (n_wk, n_k, the current doc rows) and size the
    sums from them, as the first sample of a window does."""
    K = m.K
    m.nwk.zero_()
    m.nwk[:, :K] = wk.to(m.device)
    m.nk[m.cn].zero_()
    m.nk[m.cn][:K] = nk.to(m.device)
    m.ndk[m.a].zero_()
    m.ndk[m.a][:, :K] = dk.to(m.device)
    m.T_global = int(nk.to(torch.int64).sum())
    m._ensure_avg()


def _check(m, wk, nk, dk):
    assert m._avg["wk"].dtype == torch.int64 and m._avg["dk"].dtype == torch.int64
    assert int(m._avg["k"][: m.K].min()) == S * int(nk.min())  # exact, no wrap
    m._avg["n"] = S
    m.sweeps_done = m._avg_at[-1]
    m._avg_cache = None
    th_ref, ph_ref = _reference(m, wk, nk, dk)
    th, ph = (t.cpu().to(torch.float64)[:, : m.K] for t in (m.theta(), m.phi()))
    assert bool((th > 0).all()) and bool((ph > 0).all())
    assert torch.allclose(th, th_ref, rtol=2e-6, atol=0), float(((th - th_ref) / th_ref).abs().max())
    assert torch.allclose(ph, ph_ref, rtol=2e-6, atol=0), float(((ph - ph_ref) / ph_ref).abs().max())


def _accumulate_via_apply(m, wk, nk, dk):
    """S fused applies (k_apply's acc path on a GPU, its CPU twin here) of the planted tables."""
    K, KS, V = m.K, m.KS, m.V
    _plant_tables(m, wk, nk, dk)
    ndk = m.ndk[m.a].clone()
    so = m._split_off
    d0, d1 = m.dn[0][:so], m.dn[1][:so]
    d0.zero_()
    d1.zero_()
    nk_next = torch.zeros_like(m.nk[0])
    a = m._avg
    for _ in range(S):
        ops.gibbs_apply(m.nwk, d0, d1, m.nk[m.cn], nk_next, m.q, m.qfix, V, K, KS, m.beta, m.vbeta, m.sweep_ctr,
                        bump=False, acc=(a["wk"], a["k"], a["dk"], ndk))
    assert torch.equal(a["wk"][:, :K].cpu(), wk.to(torch.int64) * S)
    assert torch.equal(a["k"][:K].cpu(), nk.to(torch.int64) * S)
    assert torch.equal(a["dk"][:, :K].cpu(), dk.to(torch.int64) * S)
    assert not bool(a["wk"][:, K:].any()) and not bool(a["dk"][:, K:].any())


def test_sums_are_int64_and_exact_cpu():
    m = _model(torch.device("cpu"))
    wk, nk, dk = _plant(m)
    _accumulate_via_apply(m, wk, nk, dk)
    _check(m, wk, nk, dk)


def test_eager_accumulate_wide_cpu():
    """Samples every post_every > 1 sweeps are added outside the graphs (GibbsLDA._accumulate)."""
    m = _model(torch.device("cpu"), sweeps=400, post_every=2)
    wk, nk, dk = _plant(m)
    _plant_tables(m, wk, nk, dk)
    for _ in range(S):
        m._accumulate()
    _check(m, wk, nk, dk)


@pytest.mark.gpu
def test_sums_are_int64_and_exact_gpu(gpu):
    m = _model(gpu)
    wk, nk, dk = _plant(m)
    _accumulate_via_apply(m, wk, nk, dk)
    _check(m, wk, nk, dk)


@pytest.mark.gpu
def test_wide_theta_phi_rows_match_narrow(gpu):
    """k_theta_rows / k_phi_rows: int64 input == the int32 kernel wherever both are exact."""
    r = np.random.default_rng(0)
    n = torch.from_numpy(r.integers(0, 2**30, (777, 24)).astype(np.int32)).to(gpu)
    nk = torch.from_numpy(r.integers(2**29, 2**30, 24).astype(np.int32)).to(gpu)
    for K in (20, 24):
        assert torch.equal(ops.theta_rows(n, K, 1.5, K * 1.5), ops.theta_rows(n.to(torch.int64), K, 1.5, K * 1.5))
        assert torch.equal(ops.phi_rows(n, nk, K, 0.5, 3.25), ops.phi_rows(n.to(torch.int64), nk.to(torch.int64), K,
                                                                              0.5, 3.25))


def test_int32_magnitude_guard(monkeypatch):
    monkeypatch.setattr(gm, "INT32_COUNT_MAX", 100)
    with pytest.raises(ValueError, match="int32 count tables"):
        _model(torch.device("cpu"))


def test_checkpoint_identity_names_the_chain(tmp_path):
    """A dense-chain checkpoint does not resume an MH run (or one with another burn-in)."""
    m = _model(torch.device("cpu"), sweeps=8)
    m.sweep(2)
    ck = Checkpointer(str(tmp_path))
    ck.save(m)
    m2 = _model(torch.device("cpu"), sweeps=8)
    m2.chain = {"sampler": "mh", "mh_burn": 20}
    with pytest.raises(ValueError, match="sampler and MH burn-in"):
        ck.restore(m2)
    m3 = _model(torch.device("cpu"), sweeps=8)
    assert ck.restore(m3) == 2


def test_checkpoint_from_before_chain_identities_resumes_dense(tmp_path):
    """A manifest / shard written before identities carried the chain (no "chain" key) is the
    dense chain: it resumes a dense run and still refuses an MH run."""
    import glob
    import json
    m = _model(torch.device("cpu"), sweeps=8)
    m.sweep(2)
    ck = Checkpointer(str(tmp_path))
    ck.save(m)
    mp = tmp_path / "manifest.json"
    man = json.loads(mp.read_text())
    man["ident"].pop("chain")
    mp.write_text(json.dumps(man))
    for f in glob.glob(str(tmp_path / "ckpt_s*.pt")):
        pl = torch.load(f, weights_only=True)
        pl["ident"].pop("chain")
        torch.save(pl, f)
    m2 = _model(torch.device("cpu"), sweeps=8)
    assert ck.restore(m2) == 2
    assert torch.equal(m2.canonical_z(), m.canonical_z())
    m3 = _model(torch.device("cpu"), sweeps=8)
    m3.chain = {"sampler": "mh", "mh_burn": 20}
    with pytest.raises(ValueError, match="sampler and MH burn-in"):
        ck.restore(m3)


def test_average_state_in_the_old_tiling_padded_format_loads():
    """Averaging sums saved KS-wide (before the K-column format) load: the padding columns are
    dropped."""
    m = _model(torch.device("cpu"), K=100)
    m.sweep(1)
    m._avg["n"] = 1
    m._accumulate()
    a = m._avg
    old = {"n": 1, "wk": a["wk"].to(torch.int64).clone(), "k": a["k"].to(torch.int64).clone(),
           "dk": a["dk"].to(torch.int64).clone()}
    assert old["wk"].shape[1] == m.KS != m.K
    want = m.average_state()
    a["wk"].fill_(-1)
    m.load_average_state(old)
    assert torch.equal(m.average_state()["wk"], want["wk"]) and torch.equal(m.average_state()["dk"], want["dk"])


def test_average_state_is_tiling_free():
    """The saved sums hold the K real topics: a KS = 112 (dense) state loads into KS = 100 (MH)."""
    m = _model(torch.device("cpu"), K=100)
    m.sweep(1)
    m._avg["n"] = 1
    m._accumulate()
    st = m.average_state()
    assert st["wk"].shape[1] == 100 and st["dk"].shape[1] == 100
    m._avg["wk"].fill_(-1)
    m.load_average_state(st)
    assert torch.equal(m._avg["wk"][:, :100], st["wk"]) and not bool(m._avg["wk"][:, 100:].any())


def test_small_counts_keep_int32_sums():
    """The default day's counts are far below 2^31 / S: the sums stay int32 (half the bytes) and
    give the same θ / φ as forced int64 sums after real sweeps."""
    out = []
    for wide in ("0", "1"):
        import os
        os.environ["ONI_POST_WIDE"] = wide
        try:
            m = _model(torch.device("cpu"), sweeps=16)
            m.sweep(16)
        finally:
            os.environ.pop("ONI_POST_WIDE", None)
        assert m._avg["wk"].dtype == (torch.int64 if wide == "1" else torch.int32)
        out.append((m.theta(), m.phi()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def test_burn_in_prefix_is_the_same_chain():
    from oni355.utils.checkpoint import _same_chain
    base = {"K": 100, "alpha": 0.5, "beta": 0.01, "seed": 1, "V": 10}
    mh = lambda b: {**base, "chain": {"sampler": "mh", "mh_burn": b}}  # noqa: E731
    assert _same_chain(mh(2), mh(3), 2)        # a 2-sweep run capped the burn-in at 2
    assert not _same_chain(mh(2), mh(3), 3)    # after its hand-over the chains differ
    assert _same_chain(mh(20), mh(20), 150)
    assert not _same_chain({**base, "chain": {"sampler": "dense", "mh_burn": 0}}, mh(20), 0)


@pytest.mark.parametrize("span,sweeps,want", [(None, 200, 50), ("0.5", 200, 50), ("0.5", 60, 30), (None, 30, 7),
                                              ("0.75", 400, 50)])
def test_post_span_caps_the_window(monkeypatch, span, sweeps, want):
    """ONI_POST_SPAN: the averaging window is at most that fraction of the chain (default the last
    quarter); ONI_POST_SAMPLES still caps the sample count."""
    if span is None:
        monkeypatch.delenv("ONI_POST_SPAN", raising=False)
    else:
        monkeypatch.setenv("ONI_POST_SPAN", span)
    m = _model(torch.device("cpu"), sweeps=sweeps)
    assert len(m._avg_at) == want and m._avg_at[-1] == sweeps
