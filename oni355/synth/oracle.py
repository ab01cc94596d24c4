"""Ground-truth recall ceiling for the synthetic days (VERDICT r5 "next round" item 2).

The generators (:mod:`oni355.synth.flow`, ``dns``, ``proxy``) export the generating label of every
row: the behaviour profile p, a long-tail behaviour ``P + b`` of the realistic day, or -1 for a
planted anomaly. With those labels the *label oracle* scores an event's token (document d, word w)
by the generative model's own form

    p*(w | d) = Σ_ℓ θ̂[d, ℓ] · P̂(w | ℓ),   θ̂[d, ℓ] = c(d, ℓ) / c(d),   P̂(w | ℓ) = c(ℓ, w) / c(ℓ)

with every count taken over the NORMAL tokens of the day (planted rows never inform it) and ℓ the
(label, token slot) pair -- a flow's source-side and destination-side words are distinct draws.
The event scores as the minimum over its tokens, as the engine's K15 score does (``k_event_min``).
Two variants:

* ``leave_in`` -- the counts include the scored event itself: the ceiling of an estimator that
  knew each document's true label mixture and each label's word distribution exactly (a planted
  word no normal label produces scores 0);
* ``loo`` -- leave-one-out: a normal event is scored with its own token removed from every count
  (a day-unique normal word then also scores 0, as it would for any estimator that learns from
  the day) -- what label knowledge alone buys from this day's data. A document with no other
  normal token falls back to the word's day marginal.
* ``loo_smooth`` -- ``loo`` with LDA's word smoothing, P̂(w | ℓ) = (c(ℓ, w) + β) / (c(ℓ) + Vβ):
  an LDA whose topic assignments are the true labels, scoring every event as the model trained
  on all the other events sees it. Day-unique words (planted or not) are then ordered by their
  documents' label mixtures, as LDA orders them.

LDA sees neither labels nor the true mixtures, so its recall is bounded by ``leave_in`` and
comparable to ``loo_smooth``. Ties count as a random order (:func:`expected_recall`).
"""
from __future__ import annotations

import numpy as np
import torch


def _dense_ids(x: torch.Tensor) -> tuple[torch.Tensor, int]:
    u, inv = torch.unique(x, return_inverse=True)
    return inv.to(torch.int64), int(u.numel())


def _lookup(keys: torch.Tensor, vals: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    """vals[i] where keys[i] == q (keys sorted ascending), 0 where q is absent."""
    if keys.numel() == 0:
        return torch.zeros(q.shape, dtype=vals.dtype, device=q.device)
    i = torch.searchsorted(keys, q).clamp_(max=keys.numel() - 1)
    hit = keys[i] == q
    return torch.where(hit, vals[i], torch.zeros((), dtype=vals.dtype, device=q.device))


def label_oracle(doc_keys: list, word_keys: list, labels: np.ndarray, device="cpu",
                 chunk: int = 1 << 21, beta: float = 0.01) -> dict:
    """Per-event oracle scores. ``doc_keys[j]`` / ``word_keys[j]``: the document / word key of
    token slot j of every event (int64-convertible arrays or tensors of length n); ``labels``:
    int [n], -1 for planted rows. Returns {"leave_in", "loo", "loo_smooth": float64 [n]}."""
    dev = torch.device(device)
    S = len(doc_keys)
    n = int(len(labels))
    lab = torch.as_tensor(np.asarray(labels, dtype=np.int64), device=dev)

    def col(k):
        t = k if torch.is_tensor(k) else torch.as_tensor(np.asarray(k))
        return t.to(device=dev, dtype=torch.int64).reshape(-1)
    d_all = torch.cat([col(k) for k in doc_keys])
    w_all = torch.cat([col(k) for k in word_keys])
    d, D = _dense_ids(d_all)
    w, V = _dense_ids(w_all)
    del d_all, w_all
    slot = torch.arange(S, device=dev).repeat_interleave(n)
    lab_t = lab.repeat(S)
    normal = lab_t >= 0
    NL = (int(lab.max()) + 1 if n else 1) * S
    lp = torch.where(normal, lab_t * S + slot, torch.full_like(lab_t, -1))
    dn, wn, ln = d[normal], w[normal], lp[normal]
    N = int(dn.numel())
    c_d = torch.bincount(dn, minlength=D).to(torch.float64)
    c_l = torch.bincount(ln, minlength=NL).to(torch.float64)
    c_w = torch.bincount(wn, minlength=V).to(torch.float64)
    dl_keys, dl_cnt = torch.unique(dn * NL + ln, return_counts=True)
    lw_keys, lw_cnt = torch.unique(ln * V + wn, return_counts=True)
    dl_cnt, lw_cnt = dl_cnt.to(torch.float64), lw_cnt.to(torch.float64)
    del dn, wn, ln
    # S(d, w) = Σ_ℓ c(d, ℓ) c(ℓ, w) / c(ℓ) for every (doc, word) pair of the day (planted included)
    pkeys, pinv = torch.unique(d * V + w, return_inverse=True)
    pd, pw = pkeys // V, pkeys % V
    dl_doc = dl_keys // NL
    lo = torch.searchsorted(dl_doc, torch.arange(D, device=dev))
    hi = torch.searchsorted(dl_doc, torch.arange(D, device=dev), right=True)
    nlab = hi - lo
    Spair = torch.zeros(pkeys.numel(), dtype=torch.float64, device=dev)
    Vb = V * beta
    Sb = torch.zeros_like(Spair)  # Σ_ℓ c(d, ℓ) c(ℓ, w) / (c(ℓ) + Vβ)
    # R(d) = Σ_ℓ c(d, ℓ) / (c(ℓ) + Vβ): the smoothing mass of a word none of d's labels produced
    R = torch.zeros(D, dtype=torch.float64, device=dev).index_add_(0, dl_doc, dl_cnt / (c_l[dl_keys % NL] + Vb))
    # expand every pair over its document's labels, in chunks of pairs (bounded memory)
    cum = torch.cumsum(nlab[pd], 0)
    start = 0
    P = pkeys.numel()
    while start < P:
        base = int(cum[start - 1]) if start else 0
        stop = int(torch.searchsorted(cum, torch.tensor(base + chunk, device=dev), right=True))
        stop = max(stop, start + 1)
        stop = min(stop, P)
        rep = nlab[pd[start:stop]]
        pid = torch.arange(start, stop, device=dev).repeat_interleave(rep)
        if pid.numel():
            first = torch.cumsum(rep, 0) - rep
            off = torch.arange(pid.numel(), device=dev) - first.repeat_interleave(rep)
            row = lo[pd[pid]] + off
            l_of = dl_keys[row] % NL
            cdl = dl_cnt[row]
            clw = _lookup(lw_keys, lw_cnt, l_of * V + pw[pid])
            Spair.index_add_(0, pid, cdl * clw / c_l[l_of])
            Sb.index_add_(0, pid, cdl * clw / (c_l[l_of] + Vb))
        start = stop
    del pd, pw
    s_tok = Spair[pinv]
    cd = c_d[d]
    marg = c_w[w] / max(N, 1)
    leave_in = torch.where(cd > 0, s_tok / cd.clamp(min=1), marg)
    # leave-one-out for normal tokens: remove the token from c(d, ℓ), c(ℓ, w), c(ℓ), c(d)
    lsafe = lp.clamp(min=0)
    cdl_own = _lookup(dl_keys, dl_cnt, d * NL + lsafe)
    clw_own = _lookup(lw_keys, lw_cnt, lsafe * V + w)
    cl_own = c_l[lsafe]
    own = cdl_own * clw_own / cl_own.clamp(min=1)
    own_loo = torch.where(cl_own > 1, (cdl_own - 1) * (clw_own - 1) / (cl_own - 1).clamp(min=1),
                          torch.zeros_like(own))
    num = s_tok - own + own_loo
    marg_loo = (c_w[w] - 1).clamp(min=0) / max(N - 1, 1)
    loo_norm = torch.where(cd > 1, num / (cd - 1).clamp(min=1), marg_loo)
    loo = torch.where(normal, loo_norm, leave_in)
    # smoothed: planted tokens (not in any count) as they are, normal ones without themselves
    sb_tok = Sb[pinv] + beta * R[d]
    sm_in = torch.where(cd > 0, sb_tok / cd.clamp(min=1), (c_w[w] + beta) / (N + Vb))
    own_b = cdl_own * clw_own / (cl_own + Vb) + beta * cdl_own / (cl_own + Vb)
    own_b_loo = (cdl_own - 1) * (clw_own - 1 + beta) / (cl_own - 1 + Vb)
    sm_loo = torch.where(cd > 1, (sb_tok - own_b + own_b_loo) / (cd - 1).clamp(min=1),
                         (c_w[w] - 1 + beta) / (N - 1 + Vb))
    loo_smooth = torch.where(normal, sm_loo, sm_in)
    out = {}
    for name, t in (("leave_in", leave_in), ("loo", loo), ("loo_smooth", loo_smooth)):
        ev = t.view(S, n).min(0).values if S > 1 else t.view(n)
        out[name] = ev.clamp(min=0).cpu().numpy()
    return out


def expected_recall(scores: np.ndarray, planted: np.ndarray, top: int) -> float:
    """Expected fraction of the planted rows in the ``top`` lowest scores when ties are ordered at
    random: a planted row with score s and n_lt rows strictly below, n_eq rows at s (itself
    included) is in with probability clip((top − n_lt) / n_eq, 0, 1)."""
    s = np.sort(scores)
    ps = scores[np.asarray(planted, dtype=np.int64)]
    n_lt = np.searchsorted(s, ps, side="left")
    n_eq = np.searchsorted(s, ps, side="right") - n_lt
    return float(np.mean(np.clip((top - n_lt) / np.maximum(n_eq, 1), 0.0, 1.0))) if ps.size else float("nan")
