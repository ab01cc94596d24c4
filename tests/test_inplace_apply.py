"""In-place apply (one process, no X01: the count pass adds Δn_wk straight into n_wk) against the
Δ-buffer apply, bitwise: auto mode across its recount → wdelta switch with a posterior
window, and a forced in-place → recount transition whose Δ heads the model must zero."""
import numpy as np
import pytest
import torch

from oni355.models import gibbs as gm
from oni355.models.corpus import build_corpus
from oni355.models.gibbs import GibbsConfig, GibbsLDA


def _model(dev, monkeypatch, inplace, **cfg):
    monkeypatch.setenv("ONI_APPLY_INPLACE", inplace)
    r = np.random.default_rng(11)
    D, V, K = 60, 40, 20
    lens = r.integers(5, 90, D)
    tdoc = np.repeat(np.arange(D), lens)
    tword = r.integers(0, V, tdoc.size)
    o = np.lexsort((tword, tdoc))
    keys = torch.arange(D, dtype=torch.int32) * 5 + 3
    c = build_corpus(torch.from_numpy(tdoc[o]).to(dev), torch.from_numpy(tword[o]).to(dev), D, V, keys.to(dev),
                     gm.tiling_for(K, "dense")[0], L=32)
    m = GibbsLDA(c, GibbsConfig(K=K, seed=9, sampler="dense", **cfg))
    assert m._inplace_ok == (inplace == "1")
    m.initialize()
    return m


def _state(m):
    s = [m.tok_z.clone(), m.nwk.clone(), m.nk_cur.clone(), m.ndk_cur.clone(), m.q.clone()]
    if m._avg is not None and m._avg["wk"] is not None:
        s += [m._avg["wk"].clone(), m._avg["k"].clone(), m._avg["dk"].clone()]
    return s


def _devices():
    out = [pytest.param("cpu")]
    out.append(pytest.param("cuda", marks=pytest.mark.gpu))
    return out


@pytest.mark.parametrize("dev", _devices())
def test_inplace_and_delta_buffer_apply_agree_across_the_auto_switch(dev, monkeypatch, request):
    if dev == "cuda":
        request.getfixturevalue("gpu")
    got = []
    for inplace in ("0", "1"):
        m = _model(torch.device(dev), monkeypatch, inplace, count_mode="auto", auto_switch=5, auto_delta="wdelta",
                   post_samples=6)
        m.plan_average(16)
        m.sweep(16)
        assert m.timings["allreduce_calls"] == 0
        got.append(_state(m))
        m.close()
    for a, b in zip(*got):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dev", _devices())
def test_recount_after_inplace_sweeps_zeroes_the_delta_heads(dev, monkeypatch, request):
    """wdelta sweeps in place, then forced recount sweeps (absolute: they need a zeroed Δ head),
    then wdelta again: equal to the same schedule with the Δ-buffer apply throughout."""
    if dev == "cuda":
        request.getfixturevalue("gpu")
    got = []
    for inplace in ("0", "1"):
        m = _model(torch.device(dev), monkeypatch, inplace, count_mode="wdelta")
        # recount (absolute, never in place: its Δ head keeps the local table), one wdelta sweep
        # (in place: it neither reads nor zeroes that head), then recount into the same buffer
        for mode, n in ((0, 1), (None, 1), (0, 2), (None, 2), (0, 1)):
            m._force_mode = mode
            if mode is None:
                m._aux_synced = False
            m.sweep(n)
        m._force_mode = None
        got.append(_state(m))
        m.check_invariants()
        m.close()
    for a, b in zip(*got):
        assert torch.equal(a, b)
