"""Scoring plans on CPU: the MFMA tile plan covers every distinct pair exactly once, and the
tile path (fma-chain numerics) agrees with the VALU pair path to within f32 rounding."""
import numpy as np
import pytest
import torch

from oni355.pipeline import common
from oni355.ref import spec


def _sides(seed, D=300, V=200, n=20_000, two=True):
    r = np.random.default_rng(seed)
    dkeys = torch.arange(D, dtype=torch.int64) * 7 + 3
    vocab = torch.arange(V, dtype=torch.int64) * 11 + 5
    mk = lambda: (dkeys[torch.from_numpy(np.minimum(r.zipf(1.4, n) - 1, D - 1))],  # noqa: E731
                  vocab[torch.from_numpy(r.integers(0, V, n))])
    return dkeys, vocab, [mk(), mk()] if two else [mk()]


def test_tile_plan_covers_every_pair_once():
    dkeys, vocab, sides = _sides(1)
    plan = common.score_plan(dkeys, vocab, sides, tiles=True)
    ref = common.score_plan(dkeys, vocab, sides, tiles=False)
    tp = plan.tiles
    assert tp is not None and plan.n_pairs == ref.n_pairs == int(tp.item_p0[-1])
    it = torch.repeat_interleave(torch.arange(tp.n_items), torch.diff(tp.item_p0))
    rc = tp.pair_rc.long()
    assert torch.equal(tp.item_docs[it * 16 + (rc >> 4)].long(), plan.pdoc.long())
    assert torch.equal(tp.item_words[it * 16 + (rc & 15)].long(), plan.pword.long())
    # same set of pairs as the doc-major plan, each event endpoint still points at its own pair
    key = lambda p: (p.pdoc.long() * 1000 + p.pword.long())  # noqa: E731
    assert torch.equal(torch.sort(key(plan))[0], key(ref))
    for a, b in zip(plan.inv, ref.inv):
        assert torch.equal(key(plan)[a.long()], key(ref)[b.long()])
    # items of one tile share their 16 documents; no column repeats a word inside an item
    w = tp.item_words.view(-1, 16)
    for i in range(tp.n_items):
        v = w[i][w[i] >= 0]
        assert v.numel() == torch.unique(v).numel()
    assert 0.0 < tp.density() <= 1.0


def test_tile_path_close_to_pair_path():
    dkeys, vocab, sides = _sides(2, two=False)
    r = np.random.default_rng(0)
    th = torch.from_numpy((r.random((300, 20)) / 20).astype(np.float32))
    ph = torch.from_numpy((r.random((200, 20)) ** 4).astype(np.float32))
    pa, pb = common.score_plan(dkeys, vocab, sides, tiles=True), common.score_plan(dkeys, vocab, sides, tiles=False)
    a = common.to_event_order(pa, common.plan_score(th, ph, pa, 1.0)[0]).numpy()
    b = common.to_event_order(pb, common.plan_score(th, ph, pb, 1.0)[0]).numpy()
    assert np.allclose(a, b, rtol=2e-6, atol=0)


@pytest.mark.parametrize("two", [False, True])
def test_event_sorted_plan_matches_event_order(two):
    """Scoring in first-endpoint pair order (SCORE_SORT_EVENTS) is a pure permutation: same
    per-event scores, same top-N rows and scores (ties by global row id) as event order."""
    dkeys, vocab, sides = _sides(3, two=two)
    r = np.random.default_rng(1)
    th = torch.from_numpy((r.random((dkeys.numel(), 20)) / 20).astype(np.float32))
    ph = torch.from_numpy((r.random((vocab.numel(), 20)) ** 4).astype(np.float32))
    ps_ = common.score_plan(dkeys, vocab, sides, tiles=False, sort_events=True)
    pu = common.score_plan(dkeys, vocab, sides, tiles=False, sort_events=False)
    assert ps_.order is not None and pu.order is None
    assert torch.equal(ps_.order[ps_.rank], torch.arange(ps_.order.numel()))
    sa, s1a, s2a = common.plan_score(th, ph, ps_, 1.0, want_parts=True)
    sb, s1b, s2b = common.plan_score(th, ph, pu, 1.0, want_parts=True)
    assert torch.equal(common.to_event_order(ps_, sa), sb)
    assert torch.equal(common.to_event_order(ps_, s1a), s1b)
    if two:
        assert torch.equal(common.to_event_order(ps_, s2a), s2b)
        assert bool((ps_.inv_sorted[0][1:] >= ps_.inv_sorted[0][:-1]).all())  # first endpoint streams
    for mr in (1, 17, 10_000):
        ra, ca = common.top_n(sa, 0.5, mr, None, row_offset=1000, order=ps_.order)
        rb, cb = common.top_n(sb, 0.5, mr, None, row_offset=1000)
        assert torch.equal(ra, rb) and torch.equal(ca, cb)


def test_fma_oracle_matches_float64_rounding():
    r = np.random.default_rng(3)
    a, b, c = (r.standard_normal(10_000).astype(np.float32) for _ in range(3))
    got = spec.fma_f32(a, b, c)
    want = (a.astype(np.float64) * b + c).astype(np.float32)  # exact product, single rounding (almost always)
    assert np.mean(got == want) > 0.999
