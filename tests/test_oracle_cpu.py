"""The label oracle (oni355.synth.oracle) against a brute-force evaluation of its definition."""
import numpy as np
import pytest

from oni355.synth.oracle import expected_recall, label_oracle


def _brute(docs, words, labels):
    S, n = len(docs), len(labels)
    toks = [(docs[j][e], words[j][e], labels[e] * S + j if labels[e] >= 0 else -1, e) for e in range(n) for j in range(S)]
    normal = [t for t in toks if t[2] >= 0]
    allw = [t[1] for t in normal]

    Vall = len({t[1] for t in toks})
    beta = 0.01

    def ps(d, w, excl=None):
        pool = [t for t in normal if not (excl is not None and t is excl)]
        cd = sum(1 for t in pool if t[0] == d)
        if cd == 0:
            return (sum(1 for t in pool if t[1] == w) + beta) / (len(pool) + Vall * beta)
        tot = 0.0
        for lab in {t[2] for t in pool if t[0] == d}:
            cdl = sum(1 for t in pool if t[0] == d and t[2] == lab)
            cl = sum(1 for t in pool if t[2] == lab)
            clw = sum(1 for t in pool if t[2] == lab and t[1] == w)
            tot += cdl / cd * (clw + beta) / (cl + Vall * beta)
        return tot

    def p(d, w, excl=None):
        pool = [t for t in normal if t[3] != excl or excl is None] if excl is not None else normal
        pool = [t for t in normal if not (excl is not None and t is excl)]
        cd = sum(1 for t in pool if t[0] == d)
        if cd == 0:
            N = len(pool)
            return sum(1 for t in pool if t[1] == w) / max(N, 1)
        tot = 0.0
        for lab in {t[2] for t in pool if t[0] == d}:
            cdl = sum(1 for t in pool if t[0] == d and t[2] == lab)
            cl = sum(1 for t in pool if t[2] == lab)
            clw = sum(1 for t in pool if t[2] == lab and t[1] == w)
            tot += cdl / cd * clw / cl
        return tot
    li = np.zeros(n)
    lo = np.zeros(n)
    sm = np.zeros(n)
    for e in range(n):
        mine = [t for t in toks if t[3] == e]
        li[e] = min(p(t[0], t[1]) for t in mine)
        lo[e] = min(p(t[0], t[1], excl=t if t[2] >= 0 else None) for t in mine)
        sm[e] = min(ps(t[0], t[1], excl=t if t[2] >= 0 else None) for t in mine)
    _ = allw
    return li, lo, sm


@pytest.mark.parametrize("S", [1, 2])
def test_label_oracle_matches_brute_force(S):
    r = np.random.default_rng(S)
    n = 120
    docs = [r.integers(0, 9, n) for _ in range(S)]
    words = [r.integers(0, 15, n) * 7 + 3 for _ in range(S)]
    labels = r.integers(0, 4, n)
    labels[r.choice(n, 6, replace=False)] = -1
    docs[0][:2] = 1000  # a document holding a single event
    got = label_oracle(docs, words, labels)
    li, lo, sm = _brute(docs, words, labels)
    np.testing.assert_allclose(got["leave_in"], li, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got["loo"], lo, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got["loo_smooth"], sm, rtol=1e-10, atol=1e-15)


def test_label_oracle_chunked_expansion_is_the_same():
    r = np.random.default_rng(7)
    n = 500
    docs, words = [r.integers(0, 30, n)], [r.integers(0, 40, n)]
    labels = r.integers(-1, 6, n)
    a = label_oracle(docs, words, labels)
    b = label_oracle(docs, words, labels, chunk=3)
    np.testing.assert_allclose(a["leave_in"], b["leave_in"], rtol=1e-13)
    np.testing.assert_allclose(a["loo"], b["loo"], rtol=1e-13)
    np.testing.assert_allclose(a["loo_smooth"], b["loo_smooth"], rtol=1e-13)


def test_expected_recall_counts_ties_fractionally():
    s = np.array([0.0, 0.0, 0.0, 0.0, 1.0, 2.0])
    assert expected_recall(s, np.array([0]), 2) == pytest.approx(0.5)
    assert expected_recall(s, np.array([4]), 5) == pytest.approx(1.0)
    assert expected_recall(s, np.array([5]), 5) == pytest.approx(0.0)
