"""Device ops: torch tensors in, torch tensors out.

CUDA (= HIP on ROCm) tensors run the hand-written gfx950 kernels of ``liboni_hip.so`` -- there is
no silent fallback, a missing library raises. CPU tensors run the NumPy specification oracle
(:mod:`oni355.ref.spec`), which is what the CPU test-suite and the ``--device cpu`` path use.

All u32 quantities (IPv4 keys, packed words, order keys) travel as ``torch.int32`` tensors holding
the same bits; kernels reinterpret them.
"""
from __future__ import annotations

import os

import ctypes as C

import numpy as np
import torch

from ..ref import spec
from . import _lib

__all__ = [
    "f32_keys", "i64_keys", "quantile_cuts", "bin_keys", "flow_keys", "flow_wordify", "sell_fill",
    "sell_perm_z", "gibbs_pass", "gibbs_apply", "mh_tables", "SAMPLER_MH", "copy_rows", "score", "select_below", "choose_tiling",
]


def _is_dev(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


def _u32np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy().view(np.uint32)


def _from_u32(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(device)


def _need(t: torch.Tensor, dtype: torch.dtype, name: str, n: int | None = None) -> None:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if n is not None and t.numel() != n:
        raise ValueError(f"{name}: expected {n} elements, got {t.numel()}")


# ------------------------------------------------------------------------------------------------
# tiling choice for the sampler: (G lanes per unit, KP topics per lane)
# ------------------------------------------------------------------------------------------------
def choose_tiling(K: int, sampler: str | None = None) -> tuple[int, int]:
    """(G, KP): lanes per sampler unit and topic slots per lane (KS = G·KP ≥ K). ``sampler`` "mh"
    (k_gibbs_mh) always runs one-lane units (S = 64 chunks a slice) with KS = K rounded up to 4."""
    if K < 1 or K > 255:
        raise ValueError("K must be in [1, 255]")
    r4 = lambda x: (x + 3) // 4 * 4  # noqa: E731
    if sampler == "mh":
        return 1, r4(K)
    if K <= 32:
        return 1, r4(K)
    wide = os.environ.get("ONI_TILING", "wide") == "wide"
    if wide and K <= 56:
        return 2, r4((K + 1) // 2)  # K = 50: 2 lanes x 28 topics (KS = 56 instead of 64)
    if K <= 48:
        return 4, 12
    if K <= 64:
        return 4, 16
    # 4-lane units up to KS = 112 (default "wide"): K = 100 pads to 112 topics instead of 128,
    # 0.848 vs 1.188 ms per 25M-token sweep on MI355X (profiles/r2s4/bench_k100_*.json);
    # ONI_TILING=narrow restores the 8-lane units above K = 64
    if wide and K <= 112:
        return 4, r4((K + 3) // 4)
    if K <= 96:
        return 8, 12
    if K <= 128:
        return 8, 16
    return 16, 16


# ------------------------------------------------------------------------------------------------
# keys / quantiles
# ------------------------------------------------------------------------------------------------
def f32_keys(x: torch.Tensor) -> torch.Tensor:
    _need(x, torch.float32, "x")
    if not _is_dev(x):
        return _from_u32(spec.f32_key(x.numpy()), x.device)
    out = torch.empty(x.numel(), dtype=torch.int32, device=x.device)
    L = _lib.lib()
    _lib.check(L.oni_f32_keys(_lib.ptr(x), x.numel(), _lib.ptr(out), _lib.stream()), "oni_f32_keys")
    return out


def i64_keys(x: torch.Tensor) -> torch.Tensor:
    _need(x, torch.int64, "x")
    if not _is_dev(x):
        return _from_u32(spec.i64_keys(x.numpy()), x.device)
    out = torch.empty(x.numel(), dtype=torch.int32, device=x.device)
    L = _lib.lib()
    _lib.check(L.oni_i64_keys(_lib.ptr(x), x.numel(), _lib.ptr(out), _lib.stream()), "oni_i64_keys")
    return out


_PASSES = ((21, 11), (10, 11), (0, 10))


def quantile_cuts(keys: torch.Tensor, fracs, allreduce=None, n_global: int | None = None) -> np.ndarray:
    """Exact cut keys at ascending ranks ceil(num*N/den)-1 (N = global count).

    ``allreduce(np.ndarray[int64]) -> np.ndarray`` sums histograms over ranks (collective X03);
    ``n_global`` is the total element count over ranks (defaults to the local count).
    """
    _need(keys, torch.int32, "keys")
    n = keys.numel() if n_global is None else int(n_global)
    dev = _is_dev(keys)
    if not dev and allreduce is None:
        return spec.quantile_cuts(_u32np(keys), fracs)
    if n == 0:
        return np.zeros(len(fracs), dtype=np.uint32)
    L = _lib.lib() if dev else None
    knp = None if dev else _u32np(keys)
    ranks = spec.quantile_ranks(n, fracs).astype(np.int64)
    prefix = np.zeros(len(fracs), dtype=np.uint64)
    hist_buf = torch.zeros(16 << 11, dtype=torch.int32, device=keys.device) if dev else None
    for shift, nbits in _PASSES:
        top = shift + nbits
        mask = 0 if top >= 32 else (0xFFFFFFFF << top) & 0xFFFFFFFF
        uniq, inv = np.unique(prefix, return_inverse=True)
        P = len(uniq)
        B = 1 << nbits
        if dev:
            pre_t = torch.from_numpy(uniq.astype(np.uint32).view(np.int32)).to(keys.device)
            hist = hist_buf[: P * B]
            hist.zero_()
            _lib.check(L.oni_radix_hist(_lib.ptr(keys), keys.numel(), shift, nbits, _lib.ptr(pre_t), P, mask,
                                        _lib.ptr(hist), _lib.stream()), "oni_radix_hist")
            if allreduce is not None and getattr(allreduce, "accepts_tensors", False):
                # X03 on the device histogram (int64: a bin's global count may pass 2^31)
                h = np.asarray(allreduce(hist.to(torch.int64) & 0xFFFFFFFF), dtype=np.int64).reshape(P, B)
            else:
                h = hist.cpu().numpy().view(np.uint32).astype(np.int64).reshape(P, B)
                if allreduce is not None:
                    h = np.asarray(allreduce(h), dtype=np.int64).reshape(P, B)
        else:
            h = spec.radix_hist(knp, shift, nbits, uniq.astype(np.uint32), mask)
            if allreduce is not None:
                h = np.asarray(allreduce(h), dtype=np.int64).reshape(P, B)
        cum = np.cumsum(h, axis=1)
        for qi in range(len(fracs)):
            c = cum[inv[qi]]
            digit = int(np.searchsorted(c, ranks[qi], side="right"))
            digit = min(digit, B - 1)
            if digit > 0:
                ranks[qi] -= c[digit - 1]
            prefix[qi] |= np.uint64(digit << shift)
    return prefix.astype(np.uint32)


def quantile_cuts_multi(keys_list: list, fracs_list: list, allreduce=None, n_global: int | None = None) -> list:
    """:func:`quantile_cuts` of several key arrays of the same length at once: each radix pass
    launches every feature's histogram, then ONE read-back (and, with ``allreduce``, one
    collective) serves them all -- 3 host round trips for a day's features instead of 3 per
    feature. Results are identical to calling :func:`quantile_cuts` per array."""
    if not keys_list:
        return []
    if not all(_is_dev(k) for k in keys_list):
        return [quantile_cuts(k, f, allreduce, n_global) for k, f in zip(keys_list, fracs_list)]
    for k in keys_list:
        _need(k, torch.int32, "keys")
    n = keys_list[0].numel() if n_global is None else int(n_global)
    if n == 0:
        return [np.zeros(len(f), dtype=np.uint32) for f in fracs_list]
    L = _lib.lib()
    dev = keys_list[0].device
    F = len(keys_list)
    ranks = [spec.quantile_ranks(n, f).astype(np.int64) for f in fracs_list]
    prefix = [np.zeros(len(f), dtype=np.uint64) for f in fracs_list]
    hist_buf = torch.zeros(F * (16 << 11), dtype=torch.int32, device=dev)
    dev_ar = allreduce is not None and getattr(allreduce, "accepts_tensors", False)
    for shift, nbits in _PASSES:
        top = shift + nbits
        mask = 0 if top >= 32 else (0xFFFFFFFF << top) & 0xFFFFFFFF
        B = 1 << nbits
        uq = [np.unique(p, return_inverse=True) for p in prefix]
        sizes = [len(u) * B for u, _ in uq]
        offs = np.concatenate([[0], np.cumsum(sizes)])
        hist = hist_buf[: offs[-1]]
        hist.zero_()
        pre_all = torch.from_numpy(np.concatenate([u for u, _ in uq]).astype(np.uint32).view(np.int32)).to(dev)
        po = np.concatenate([[0], np.cumsum([len(u) for u, _ in uq])])
        for f in range(F):
            _lib.check(L.oni_radix_hist(_lib.ptr(keys_list[f]), keys_list[f].numel(), shift, nbits,
                                        pre_all.data_ptr() + 4 * int(po[f]), len(uq[f][0]), mask,
                                        hist.data_ptr() + 4 * int(offs[f]), _lib.stream()), "oni_radix_hist")
        if dev_ar:
            h_all = np.asarray(allreduce(hist.to(torch.int64) & 0xFFFFFFFF), dtype=np.int64)
        else:
            h_all = hist.cpu().numpy().view(np.uint32).astype(np.int64)
            if allreduce is not None:
                h_all = np.asarray(allreduce(h_all), dtype=np.int64)
        for f in range(F):
            uniq, inv = uq[f]
            cum = np.cumsum(h_all[offs[f]:offs[f + 1]].reshape(len(uniq), B), axis=1)
            for qi in range(len(fracs_list[f])):
                c = cum[inv[qi]]
                digit = min(int(np.searchsorted(c, ranks[f][qi], side="right")), B - 1)
                if digit > 0:
                    ranks[f][qi] -= c[digit - 1]
                prefix[f][qi] |= np.uint64(digit << shift)
    return [p.astype(np.uint32) for p in prefix]


def quantile_cuts_dev(keys_list: list, fracs_list: list, allreduce_=None, n_global: int | None = None) -> torch.Tensor:
    """:func:`quantile_cuts_multi` without a host round trip: every pass's histograms, the
    (optional, device) all-reduce ``allreduce_(tensor)`` and the digit pick (k_quantile_pick) stay
    on the stream; returns the concatenated cuts of all features as a device int32 tensor (u32
    bits), ready for the wordify kernels. Same cuts as :func:`quantile_cuts_multi`."""
    for k in keys_list:
        _need(k, torch.int32, "keys")
    dev = keys_list[0].device
    n = keys_list[0].numel() if n_global is None else int(n_global)
    nq = [len(f) for f in fracs_list]
    NQ = int(sum(nq))
    if n == 0:  # an empty day: all-zero cuts, as quantile_cuts_multi
        return torch.zeros(NQ, dtype=torch.int32, device=dev)
    ranks = np.concatenate([spec.quantile_ranks(n, f).astype(np.int64) for f in fracs_list])
    qoff = np.concatenate([[0], np.cumsum(nq)]).astype(np.int64)
    B = 1 << 11
    hoff = qoff * B  # feature f's histograms start at hoff[f]
    # histogram of query q in a pass of b bits: pass 1 one shared histogram per feature (every
    # prefix is 0), later passes one per query at q_local << b inside the feature's region
    bases_np = [np.concatenate([np.full(nq[f], hoff[f]) for f in range(len(nq))])]
    for _, nbits in _PASSES[1:]:
        bases_np.append(np.concatenate([hoff[f] + (np.arange(nq[f]) << nbits) for f in range(len(nq))]))
    # one pinned upload (non-blocking: a pageable copy would wait for the whole queue)
    host = torch.empty(NQ * 2 + NQ * len(_PASSES), dtype=torch.int32, pin_memory=dev.type == "cuda")
    hv = host.numpy()
    hv[: 2 * NQ] = ranks.view(np.int32)
    for i, b_ in enumerate(bases_np):
        hv[(2 + i) * NQ: (3 + i) * NQ] = b_.astype(np.int32)
    st = host.to(dev, non_blocking=True)
    rank = st[: 2 * NQ].view(torch.int64)
    bases = [st[(2 + i) * NQ: (3 + i) * NQ] for i in range(len(_PASSES))]
    prefix = torch.zeros(NQ, dtype=torch.int32, device=dev)
    hist = torch.empty(int(hoff[-1]), dtype=torch.int32, device=dev)
    L = _lib.lib()
    for pi, (shift, nbits) in enumerate(_PASSES):
        top = shift + nbits
        mask = 0 if top >= 32 else (0xFFFFFFFF << top) & 0xFFFFFFFF
        hist.zero_()
        for f, k in enumerate(keys_list):
            P = 1 if pi == 0 else nq[f]
            _lib.check(L.oni_radix_hist(_lib.ptr(k), k.numel(), shift, nbits, prefix.data_ptr() + 4 * int(qoff[f]), P,
                                        mask, hist.data_ptr() + 4 * int(hoff[f]), _lib.stream()), "oni_radix_hist")
        if allreduce_ is not None:
            allreduce_(hist)
        _lib.check(L.oni_quantile_pick(_lib.ptr(hist), _lib.ptr(bases[pi]), NQ, nbits, shift,
                                       _lib.ptr(prefix), _lib.ptr(rank), _lib.stream()), "oni_quantile_pick")
    return prefix


def bin_keys(keys: torch.Tensor, cuts: np.ndarray) -> torch.Tensor:
    _need(keys, torch.int32, "keys")
    if not _is_dev(keys):
        return torch.from_numpy(spec.bin_keys(_u32np(keys), cuts))
    c = _from_u32(np.asarray(cuts, dtype=np.uint32), keys.device)
    out = torch.empty(keys.numel(), dtype=torch.uint8, device=keys.device)
    _lib.check(_lib.lib().oni_bin_keys(_lib.ptr(keys), keys.numel(), _lib.ptr(c), len(cuts), _lib.ptr(out),
                                       _lib.stream()), "oni_bin_keys")
    return out


# ------------------------------------------------------------------------------------------------
# flow featurization
# ------------------------------------------------------------------------------------------------
def flow_keys(hour, minute, second, ibyt, ipkt):
    n = hour.numel()
    for t, nm, dt in ((hour, "hour", torch.int32), (minute, "minute", torch.int32), (second, "second", torch.int32),
                      (ibyt, "ibyt", torch.int64), (ipkt, "ipkt", torch.int64)):
        _need(t, dt, nm, n)
    if not _is_dev(hour):
        tk, bk, pk = spec.flow_keys(hour.numpy(), minute.numpy(), second.numpy(), ibyt.numpy(), ipkt.numpy())
        return tuple(_from_u32(x, hour.device) for x in (tk, bk, pk))
    outs = [torch.empty(n, dtype=torch.int32, device=hour.device) for _ in range(3)]
    _lib.check(_lib.lib().oni_flow_keys(*map(_lib.ptr, (hour, minute, second, ibyt, ipkt)), n,
                                        *map(_lib.ptr, outs), _lib.stream()), "oni_flow_keys")
    return tuple(outs)


def flow_wordify(sport, dport, tkey, bkey, pkey, tcuts, bcuts, pcuts, dev_cuts: torch.Tensor | None = None):
    """Flow words (K03). ``dev_cuts``: the three cut arrays already on the device, concatenated
    (from :func:`quantile_cuts_dev`); ``tcuts``/``bcuts``/``pcuts`` then only give the counts."""
    n = sport.numel()
    _need(sport, torch.int32, "sport", n)
    _need(dport, torch.int32, "dport", n)
    for t, nm in ((tkey, "tkey"), (bkey, "bkey"), (pkey, "pkey")):
        _need(t, torch.int32, nm, n)
    if not _is_dev(sport):
        sw, dw = spec.flow_wordify(sport.numpy(), dport.numpy(), _u32np(tkey), _u32np(bkey), _u32np(pkey),
                                   tcuts, bcuts, pcuts)
        return _from_u32(sw, sport.device), _from_u32(dw, sport.device)
    if dev_cuts is not None:
        if dev_cuts.numel() != len(tcuts) + len(bcuts) + len(pcuts) or dev_cuts.dtype != torch.int32:
            raise ValueError("flow_wordify: device cuts must be the int32 concatenation of the three cut arrays")
        c = dev_cuts
    else:
        cuts = np.concatenate([np.asarray(tcuts, np.uint32), np.asarray(bcuts, np.uint32),
                               np.asarray(pcuts, np.uint32)])
        c = _from_u32(cuts, sport.device)
    sw = torch.empty(n, dtype=torch.int32, device=sport.device)
    dw = torch.empty(n, dtype=torch.int32, device=sport.device)
    _lib.check(_lib.lib().oni_flow_wordify(_lib.ptr(sport), _lib.ptr(dport), _lib.ptr(tkey), _lib.ptr(bkey),
                                           _lib.ptr(pkey), n, _lib.ptr(c), len(tcuts), len(bcuts), len(pcuts),
                                           _lib.ptr(sw), _lib.ptr(dw), _lib.stream()), "oni_flow_wordify")
    return sw, dw


# ------------------------------------------------------------------------------------------------
# SELL layout
# ------------------------------------------------------------------------------------------------
def sell_fill(chunk_doc, chunk_pos0, chunk_len, S, slice_off, doc_pair_ptr, pair_tokoff, pair_word, pair_cnt,
              tok_word):
    if not _is_dev(tok_word):
        tw = tok_word.numpy().view(np.uint32)
        spec.sell_fill(chunk_doc.numpy(), chunk_pos0.numpy(), chunk_len.numpy(), S, slice_off.numpy(),
                       doc_pair_ptr.numpy(), pair_tokoff.numpy(), pair_word.numpy(), pair_cnt.numpy(), tw)
        return tok_word
    _need(chunk_doc, torch.int32, "chunk_doc")
    _need(slice_off, torch.int64, "slice_off")
    _need(pair_tokoff, torch.int64, "pair_tokoff")
    _lib.check(_lib.lib().oni_sell_fill(*map(_lib.ptr, (chunk_doc, chunk_pos0, chunk_len)), chunk_doc.numel(), S,
                                        *map(_lib.ptr, (slice_off, doc_pair_ptr, pair_tokoff, pair_word, pair_cnt,
                                                        tok_word)), _lib.stream()), "oni_sell_fill")
    return tok_word


def sell_perm_z(chunk_doc, chunk_pos0, chunk_len, S, slice_off, doc_tok_ptr, tok_z, canon_z, to_canon: bool):
    if not _is_dev(tok_z):
        cd, cp, cl, so, dt = (x.numpy() for x in (chunk_doc, chunk_pos0, chunk_len, slice_off, doc_tok_ptr))
        tz, cz = tok_z.numpy(), canon_z.numpy()
        for i in np.nonzero(cd >= 0)[0]:
            off = int(so[i // S]) + i % S
            sidx = off + np.arange(int(cl[i])) * S
            base = int(dt[cd[i]]) + int(cp[i])
            if to_canon:
                cz[base:base + int(cl[i])] = tz[sidx]
            else:
                tz[sidx] = cz[base:base + int(cl[i])]
        return
    _lib.check(_lib.lib().oni_sell_perm_z(*map(_lib.ptr, (chunk_doc, chunk_pos0, chunk_len)), chunk_doc.numel(), S,
                                          _lib.ptr(slice_off), _lib.ptr(doc_tok_ptr), _lib.ptr(tok_z),
                                          _lib.ptr(canon_z), 0 if to_canon else 1, _lib.stream()),
               "oni_sell_perm_z")


# ------------------------------------------------------------------------------------------------
# sampler
# ------------------------------------------------------------------------------------------------
SAMPLER_MH = 4


def gibbs_pass(st: dict, G: int, KP: int, K: int, alpha: float, seed: int, init: bool, sweep_ctr: torch.Tensor,
               chunk_len: torch.Tensor, host_sweep: int | None = None, mode: int = 1,
               sampler: int = 0, chg_mask: torch.Tensor | None = None, wpos: torch.Tensor | None = None,
               z_w: torch.Tensor | None = None, zz_w: torch.Tensor | None = None,
               alpha_in_row: bool = False, mh_doc_moves: int = 1, word_init: bool = False,
               pos_aligned: bool = False) -> None:
    """Launch one init/sweep pass. ``st`` holds the OniGibbs tensors (csrc/kernels/gibbs_sampler.h);
    sweeps also need ``st["qfix"]`` ([2, KS] f32, from :func:`gibbs_apply`).

    ``mode`` 1: accumulate Δn_wk with per-token atomics; 0: the caller rebuilds n_wk with
    :func:`recount`; 2: record changed slots in ``chg_mask`` for :func:`delta_recount`; 3: also
    write changed topics into the word-sorted copy ``z_w`` (via ``wpos``) for a streaming recount;
    4: changed tokens set their word-sorted bit in ``chg_mask`` (int32 bitmap) and record
    old | new << 8 in the low half of ``zz_w`` (int32 [T], word-sorted, from :func:`wdelta_records`)
    for :func:`wdelta_recount`.
    ``sampler`` (kernel variant; every variant draws the same topics bit for bit): 0 = generic
    k_gibbs, 2 = k_gibbs_ldsg (G > 1), 3 = k_gibbs_x1 (G = 1); the specialised kernels need
    ``alpha_in_row`` (n + α exact in f32 for every count of the corpus), else the generic one runs.
    4 = k_gibbs_mh, the Metropolis-Hastings sampler (one-lane units, chunks ≤ 127 tokens; NOT the
    same draws: its own oracle spec.gibbs_pass_mh) which also needs the word proposal
    (``st["walias"]`` + ``st["wsum"]``, or ``st["wcdf"]``), ``st["dalias"]``, ``st["mh_g"]``
    (:func:`mh_tables`) and ``st["chunk_dslot"]``;
    ``mh_doc_moves`` doc moves after each token's word move.
    """
    s0, s1 = spec.split_seed(seed)
    KS = G * KP
    nk_rep = st["dnk"].numel() // KS
    if nk_rep < 1 or nk_rep * KS != st["dnk"].numel() or nk_rep & (nk_rep - 1):
        raise ValueError("dnk must hold a power-of-two number of [KS] replicas")
    if not init and (st.get("qfix") is None or st["qfix"].numel() != 2 * KS):
        raise ValueError("a sweep needs the [2, KS] token-exclusion table qfix")
    if mode == 4:
        T = int(zz_w.numel()) if zz_w is not None else 0
        if (wpos is None or zz_w is None or chg_mask is None or wpos.numel() != st["tok_word"].numel()
                or zz_w.dtype != torch.int32 or chg_mask.dtype != torch.int32 or chg_mask.numel() * 32 < T):
            raise ValueError("wdelta mode needs wpos [SELL slots], int32 zz_w [T] and an int32 bitmap of T bits")
    if not _is_dev(st["tok_word"]):
        chg = st.get("chg_count")
        z_before = st["tok_z"].clone() if (chg is not None or mode == 4) else None
        npst = {k: (v.numpy().view(np.uint32) if k in ("tok_word", "chunk_key", "walias", "dalias") else v.numpy())
                for k, v in st.items() if isinstance(v, torch.Tensor)}
        npst["dnk"] = npst["dnk"][:KS]  # replica 0 (the sum over replicas is what counts)
        if mode != 1:
            npst["dnwk"] = np.zeros_like(npst["dnwk"])  # discarded: recount rebuilds n_wk
        if not init:
            npst["qfix"] = npst["qfix"].reshape(2, KS)
        sweep_no = int(host_sweep if host_sweep is not None else sweep_ctr.item())
        if sampler == SAMPLER_MH and not init:
            if G != 1:
                raise ValueError("the MH sampler runs one-lane units")
            if st.get("tok_zlag") is not None:
                raise ValueError("the lagged word side (ONI_X01_LAG) runs the dense samplers only")
            spec.gibbs_pass_mh(npst, KS, K, alpha, s0, s1, sweep_no, chunk_len.numpy(), doc_moves=mh_doc_moves)
        else:
            spec.gibbs_pass(npst, G, KP, K, alpha, s0, s1, init, sweep_no, chunk_len.numpy(), word_init=word_init)
        if mode == 3:
            valid = wpos >= 0
            z_w[wpos[valid].long()] = st["tok_z"][valid]
        if mode == 4:
            ch = st["tok_z"] != z_before
            p = wpos[ch].long()
            zz16 = (z_before[ch].to(torch.int32) | (st["tok_z"][ch].to(torch.int32) << 8))
            zz_w.view(torch.int16).view(-1, 2)[p, 0] = torch.where(zz16 >= 0x8000, zz16 - 0x10000, zz16).to(torch.int16)
            upd = np.zeros(chg_mask.numel(), dtype=np.uint32)
            np.bitwise_or.at(upd, (p >> 5).numpy(), (np.uint32(1) << (p & 31).numpy().astype(np.uint32)))
            chg_mask |= torch.from_numpy(upd.view(np.int32))
        if chg is not None:
            chg += int((st["tok_z"] != z_before).sum())
        return
    n_slices = st["slice_len"].numel()
    if st["q"].shape[-1] != KS or st["ndk_src"].shape[-1] != KS:
        raise ValueError("q / ndk row width must equal G*KP")
    if st["chunk_doc"].numel() != n_slices * (64 // G):
        raise ValueError("chunk table must hold S chunks per slice")
    a = _lib.OniGibbs()
    for name in ("tok_word", "tok_z", "slice_off", "slice_len", "chunk_doc", "chunk_pos0", "chunk_key",
                 "chunk_multi", "ndk_src", "ndk_dst", "q", "dnwk", "dnk"):
        setattr(a, name, _lib.ptr(st[name]))
    if not init:
        a.qfix = _lib.ptr(st["qfix"])
    a.sweep_ctr = _lib.ptr(sweep_ctr)
    if mode == 2:
        if chg_mask is None or chg_mask.numel() * (64 // G) < st["tok_word"].numel():
            raise ValueError("delta mode needs a change mask with one word per SELL step")
        a.chg_mask = _lib.ptr(chg_mask)
    if mode == 3:
        if wpos is None or z_w is None or wpos.numel() != st["tok_word"].numel():
            raise ValueError("dual mode needs wpos [SELL slots] and z_w [T]")
        a.wpos, a.z_w = _lib.ptr(wpos), _lib.ptr(z_w)
    if mode == 4:
        a.wpos, a.zz_w, a.chg_mask = _lib.ptr(wpos), _lib.ptr(zz_w), _lib.ptr(chg_mask)
    if st.get("chg_count") is not None:
        a.chg_count = _lib.ptr(st["chg_count"])
    if not init and st.get("exact_guard") is not None:
        a.exact_guard = _lib.ptr(st["exact_guard"])
    if not init and st.get("tok_zlag") is not None:
        if sampler == SAMPLER_MH:
            raise ValueError("the lagged word side (ONI_X01_LAG) runs the dense samplers only")
        if st["tok_zlag"].numel() != st["tok_z"].numel() or st["tok_zlag"].dtype != torch.uint8:
            raise ValueError("tok_zlag must be a uint8 SELL array like tok_z")
        a.tok_zlag = _lib.ptr(st["tok_zlag"])
    a.n_slices, a.K, a.KS, a.alpha, a.seed0, a.seed1 = n_slices, K, KS, float(alpha), s0, s1
    a.nk_rep = nk_rep
    # the caller vouches that n + α is exact in f32 for every doc-topic count of this corpus
    # ONI_SAMPLER_AB (kernel A/B, bench/sampler_ab.py): bit 0 = word-sorted slots loaded on change
    # (k_gibbs_x1), bit 1 = 4-wave register budget (k_gibbs_ldsg)
    # pos_aligned: every chunk starts at a multiple of 4 tokens (chunk length % 4 == 0), so the
    # one-lane sampler picks its Philox word by the uniform step index (bit 4)
    ab = int(os.environ.get("ONI_SAMPLER_AB", "0"))
    # bit 2 of ONI_SAMPLER_AB (flags bit 5): k_gibbs_x1's q' by v_pk_fma_f32 on topic pairs (A/B: loses);
    # bit 3 (flags bit 7): its ±1 count update by per-topic bfe + cvt instead of the LDS table (A/B);
    # bit 5 (flags bit 9): k_gibbs_mh's round-5 level-1 word CDF gathers (one lane per row, words two
    # tokens ahead) instead of four lanes per row a step ahead (A/B)
    a.flags = ((1 if alpha_in_row else 0) | (ab & 3) << 1 | (8 if (init and word_init) else 0)
               | (16 if pos_aligned else 0) | (32 if ab & 4 else 0) | (128 if ab & 8 else 0)
               | (512 if ab & 32 else 0))
    if sampler == SAMPLER_MH:
        if G != 1:
            raise ValueError("the MH sampler runs one-lane units")
        m = _lib.OniMH()
        m.g = a
        m.chunk_len = _lib.ptr(chunk_len)
        m.lmax = int(st["mh_lmax"])
        m.kalpha = float(np.float32(K) * np.float32(alpha))
        m.inv_alpha = float(np.float32(1.0 / alpha))
        m.doc_moves = int(mh_doc_moves)
        if not init:
            for name in ("dalias", "chunk_dslot"):
                setattr(m, name, _lib.ptr(st[name]))
            if st.get("wcdf") is not None:
                m.wcdf, m.wp = _lib.ptr(st["wcdf"]), (8 if K <= 128 else 16)
            else:
                m.walias, m.wsum, m.wp = _lib.ptr(st["walias"]), _lib.ptr(st["wsum"]), 0
            m.mh_g = _lib.ptr(st["mh_g"])
        _lib.check(_lib.lib().oni_gibbs_mh_launch(C.byref(m), 1 if init else 0, int(mode), _lib.stream()),
                   "oni_gibbs_mh_launch")
        return
    _lib.check(_lib.lib().oni_gibbs_launch(C.byref(a), G, KP, 1 if init else 0, int(mode), int(sampler),
                                           _lib.stream()), "oni_gibbs_launch")


def mh_tables(q: torch.Tensor, nk: torch.Tensor, ndk_src: torch.Tensor, long_rows: torch.Tensor, K: int,
              alpha: float, vbeta: float, dalias: torch.Tensor, g: torch.Tensor, walias: torch.Tensor | None = None,
              wsum: torch.Tensor | None = None, wcdf: torch.Tensor | None = None) -> None:
    """Per-sweep tables of the MH sampler (spec.mh_tables). Word proposal ∝ q[w, ·], one of:
    ``walias`` [V, K, 4] := every word's alias records {entry, q_j, q_alias, Σ q} and ``wsum`` [V]
    its sums (k_mh_alias), or ``wcdf`` [V, 16] f32 := its level-1 CDF row (k_mh_cdf). ``dalias``
    [n_long, K] := the alias entries of n_dk + α for every document over several chunks (rows
    ``long_rows`` of ``ndk_src``), ``g`` [KS] := 1/(n_k + Vβ + 1) of the snapshot's topic totals
    ``nk``. int32 tensors hold the u32 entries."""
    cdf = wcdf is not None
    if cdf == (walias is not None) or (walias is not None and wsum is None):
        raise ValueError("one word proposal table: walias + wsum, or wcdf")
    if cdf and (wcdf.shape != (q.shape[0], spec.MH_CDF_BUCKETS) or wcdf.dtype != torch.float32):
        raise ValueError("wcdf must be a [V, 16] float32 table")
    if not _is_dev(q):
        wt, ws, da, gg = spec.mh_tables(q.numpy(), nk.numpy(), ndk_src.numpy(), long_rows.numpy(), K, alpha, vbeta,
                                        word="cdf" if cdf else "alias")
        if cdf:
            wcdf.copy_(torch.from_numpy(wt))
        else:
            walias.copy_(torch.from_numpy(wt.view(np.int32)))
            wsum.copy_(torch.from_numpy(ws))
        if da.shape[0]:
            dalias.copy_(torch.from_numpy(da.view(np.int32)))
        g.copy_(torch.from_numpy(gg))
        return
    V, KS = q.shape
    p = lambda t: _lib.ptr(t) if t is not None else None  # noqa: E731
    _lib.check(_lib.lib().oni_mh_tables(_lib.ptr(q), V, K, KS, _lib.ptr(ndk_src), _lib.ptr(long_rows),
                                        long_rows.numel(), float(alpha), p(walias), p(wsum), p(wcdf),
                                        _lib.ptr(dalias), _lib.ptr(nk), float(vbeta), _lib.ptr(g), _lib.stream()),
               "oni_mh_tables")


def delta_recount(wslot, tile_wlo, tile_whi, chg_mask, tok_word, tok_z, tok_zprev, dnwk_out, KS: int, G: int) -> None:
    """Δn_wk of the tokens whose topic changed this sweep (+1 new, -1 previous); refreshes z_prev."""
    T = wslot.numel()
    if T == 0:
        return
    if not _is_dev(tok_z):
        sl = wslot.long()
        zn, zo = tok_z[sl].long(), tok_zprev[sl].long()
        ch = zn != zo
        w = tok_word[sl][ch].long()
        one = torch.ones(int(ch.sum()), dtype=torch.int32)
        dnwk_out.view(-1).index_add_(0, w * KS + zn[ch], one)
        dnwk_out.view(-1).index_add_(0, w * KS + zo[ch], -one)
        tok_zprev[sl[ch]] = tok_z[sl[ch]]
        return
    S = 64 // G
    wmax = max(1, RECOUNT_CELLS // KS)  # small LDS histograms: occupancy, not capacity, bounds these kernels
    _lib.check(_lib.lib().oni_delta_recount(*map(_lib.ptr, (wslot, tile_wlo, tile_whi, chg_mask, tok_word, tok_z,
                                                            tok_zprev)), T, _lib.ptr(dnwk_out), KS,
                                            S.bit_length() - 1, G, RECOUNT_TILE, wmax, _lib.stream()),
               "oni_delta_recount")


WBITS_BLOCK = 8192  # word-sorted positions per k_wdelta_recount block (matches kWBitsPerBlock)


def wdelta_records(wsorted: torch.Tensor) -> torch.Tensor:
    """The int32 [T] record array of MODE 4: high half = each position's word minus the first word
    of its k_wdelta_recount block (0xFFFF when that does not fit), low half = the (old | new << 8)
    topics the sampler writes for a changed token (zero here)."""
    T = wsorted.numel()
    out = torch.zeros((max(T, 1), 2), dtype=torch.int16, device=wsorted.device)
    if T:
        nb = -(-T // WBITS_BLOCK)
        w = torch.nn.functional.pad(wsorted.to(torch.int32), (0, nb * WBITS_BLOCK - T)).view(nb, WBITS_BLOCK)
        rel = (w - w[:, :1]).view(-1)[:T].clamp_(max=0xFFFF)  # word-sorted: ≥ 0
        out[:T, 1] = torch.where(rel >= 0x8000, rel - 0x10000, rel).to(torch.int16)
    return out.view(torch.int32).view(-1)


def wdelta_recount(wbits, wsorted, zz_w, dnwk_out, KS: int) -> None:
    """Δn_wk of the tokens marked in the word-sorted bitmap ``wbits`` (+1 at (w, new), -1 at
    (w, old) with zz_w's low half = old | new << 8, its high half the row in the block: see
    :func:`wdelta_records`); clears the bitmap (k_wdelta_recount)."""
    T = wsorted.numel()
    if T == 0:
        return
    if not _is_dev(wsorted):
        b = wbits.numpy().view(np.uint32)
        pos = np.nonzero(np.unpackbits(b.view(np.uint8), bitorder="little")[:T])[0]
        pt = torch.from_numpy(pos)
        w = wsorted[pt].long()
        one = torch.ones(pos.size, dtype=torch.int32)
        zz = zz_w[pt].to(torch.int64) & 0xFFFF
        dnwk_out.view(-1).index_add_(0, w * KS + (zz >> 8), one)
        dnwk_out.view(-1).index_add_(0, w * KS + (zz & 0xFF), -one)
        wbits.zero_()
        return
    if zz_w.dtype != torch.int32 or zz_w.numel() < T:
        raise ValueError("zz_w must be the int32 [T] record array of wdelta_records")
    wmax = max(1, RECOUNT_CELLS // KS)
    _lib.check(_lib.lib().oni_wdelta_recount(*map(_lib.ptr, (wbits, wsorted, zz_w)), T, _lib.ptr(dnwk_out), KS,
                                             wmax, _lib.stream()), "oni_wdelta_recount")


RECOUNT_TILE = 4096
DN_AUX = 4  # auxiliary int32 words at the end of a Δ buffer (matches kDnAux)
RECOUNT_CELLS = 2048  # LDS histogram cells per recount block (8 KB; matches kRecountCells)


def exact_guard(ndk: torch.Tensor, rows: torch.Tensor, K: int, limit: int, flag: torch.Tensor) -> None:
    """flag[0] := 1 if every count of ``rows`` (first K columns of ``ndk``) is ≤ ``limit``, else 0
    (k_exact_guard: the row-f32 samplers run this sweep only when it is 1)."""
    KS = ndk.shape[-1]
    if not _is_dev(ndk):
        ok = not bool((ndk[rows.long(), :K] > limit).any()) if rows.numel() else True
        flag.fill_(1 if ok else 0)
        return
    _lib.check(_lib.lib().oni_exact_guard(_lib.ptr(ndk), _lib.ptr(rows), int(rows.numel()), KS, K, int(limit),
                                          _lib.ptr(flag), _lib.stream()), "oni_exact_guard")


def recount(wsorted, wslot, tok_z, nwk_out, KS: int) -> None:
    """Accumulate the (word, topic) histogram of all tokens into ``nwk_out`` [V, KS] (pre-zeroed).

    ``wslot`` maps word-sorted tokens to SELL slots of ``tok_z``; ``wslot=None`` means ``tok_z``
    is already in word-sorted order (the streaming recount of the dual-z mode).
    """
    T = wsorted.numel()
    if T == 0:
        return
    if not _is_dev(tok_z):
        z = (tok_z[wslot.long()] if wslot is not None else tok_z[:T]).long()
        nwk_out.view(-1).index_add_(0, wsorted.long() * KS + z, torch.ones_like(z, dtype=torch.int32))
        return
    wmax = max(1, RECOUNT_CELLS // KS)  # small LDS histograms: occupancy, not capacity, bounds these kernels
    if wslot is None and KS <= 32 and STREAM_RECOUNT:
        # word-sorted topics: contiguous per-thread runs counted in registers (k_recount_reg)
        _lib.check(_lib.lib().oni_recount_stream(_lib.ptr(wsorted), _lib.ptr(tok_z), T, _lib.ptr(nwk_out), KS,
                                                 RECOUNT_TILE, wmax, _lib.stream()), "oni_recount_stream")
        return
    _lib.check(_lib.lib().oni_recount(_lib.ptr(wsorted), _lib.ptr(wslot), _lib.ptr(tok_z), T, _lib.ptr(nwk_out), KS,
                                      RECOUNT_TILE, wmax, _lib.stream()), "oni_recount")


STREAM_RECOUNT = True  # k_recount_reg (register runs) 0.065 ms vs k_recount (LDS) 0.093 ms, both at 8 KB LDS


def gibbs_apply(nwk, dcur, dother, nk_cur, nk_next, q, qfix, V, K, KS, beta, vbeta, sweep_ctr, bump=True,
                absolute=False, rows_copy=None, acc=None, inplace=False):
    """n_wk ← Δ (or absolute), n_k ← n_k + Σ_replicas Δn_k, q refresh (+ the token-exclusion
    table ``qfix`` [2, KS]); zeroes ``dother``.

    ``dcur``/``dother`` are [V·KS + R·KS + DN_AUX]: the Δn_wk table, R replicas of Δn_k, then
    DN_AUX auxiliary words ([0] = tokens that changed topic; all-reduced with the rest).
    ``rows_copy = (src, dst, rows)``: also :func:`copy_rows` in the same launch.
    ``acc = (wk, k, dk, ndk)``: the posterior-average sums [V, KS], [KS], [D, KS] (each int32 or
    int64) also gain the new n_wk, n_k and the doc rows ``ndk`` [D, KS] (int32) in the same launch.
    ``inplace``: this sweep's Δn_wk is already in ``nwk`` (the count pass wrote it there: one process,
    no X01); the Δ heads of ``dcur`` / ``dother`` are neither read nor zeroed."""
    if inplace and absolute:
        raise ValueError("an absolute (recount) sweep cannot apply in place")
    if acc is not None:
        wk, kk, dk, ndk = acc
        if (any(t.dtype not in (torch.int32, torch.int64) for t in (wk, kk, dk))
                or tuple(wk.shape) != (V, KS) or kk.numel() != KS or tuple(dk.shape) != tuple(ndk.shape)
                or ndk.dtype != torch.int32 or ndk.shape[-1] != KS):
            raise ValueError("posterior sums must be int32/int64 [V, KS], [KS], [D, KS] over int32 [D, KS] doc rows")
    nk_rep = (dcur.numel() - V * KS - DN_AUX) // KS
    if nk_rep < 1 or V * KS + nk_rep * KS + DN_AUX != dcur.numel():
        raise ValueError("Δ buffer must be [V*KS + nk_rep*KS + DN_AUX]")
    if qfix.numel() != 2 * KS or qfix.dtype != torch.float32:
        raise ValueError("qfix must be a [2, KS] float32 table")
    if not _is_dev(nwk):
        base = np.zeros_like(nwk.numpy()) if absolute else nwk.numpy()
        head = torch.zeros(V, KS, dtype=torch.int32) if inplace else dcur[: V * KS].view(V, KS)
        n2, nk2, q2, qf = spec.gibbs_apply(base, head.numpy(),
                                           dcur[V * KS: V * KS + nk_rep * KS].view(-1, KS).sum(0, dtype=torch.int32).numpy(),
                                           nk_cur.numpy(), K, beta, vbeta)
        nwk.copy_(torch.from_numpy(n2))
        nk_next.copy_(torch.from_numpy(nk2))
        q.copy_(torch.from_numpy(q2))
        qfix.copy_(torch.from_numpy(qf).view_as(qfix))
        if inplace:
            dother[V * KS:].zero_()
        else:
            dother.zero_()
        if bump:
            sweep_ctr += 1
        if rows_copy is not None:
            copy_rows(*rows_copy, KS)
        if acc is not None:
            wk += nwk
            kk += nk_next
            dk += ndk
        return
    rs, rd, rr = rows_copy if rows_copy is not None and rows_copy[2].numel() else (None, None, None)
    aw = ak = ad = an = None
    wide = 0
    if acc is not None:
        aw, ak, ad, an = (_lib.ptr(t) for t in acc)
        wide = sum(b for b, t in ((1, acc[0]), (2, acc[1]), (4, acc[2])) if t.dtype == torch.int64)
    _lib.check(_lib.lib().oni_gibbs_apply(*map(_lib.ptr, (nwk, dcur, dother, nk_cur, nk_next, q, qfix)), V, K, KS,
                                          float(beta), float(vbeta), _lib.ptr(sweep_ctr), 1 if bump else 0,
                                          1 if absolute else 0, nk_rep, _lib.ptr(rs) if rs is not None else None,
                                          _lib.ptr(rd) if rd is not None else None,
                                          _lib.ptr(rr) if rr is not None else None, rr.numel() if rr is not None else 0,
                                          aw, ak, ad, wide, an, acc[3].shape[0] if acc is not None else 0,
                                          1 if inplace else 0, _lib.stream()), "oni_gibbs_apply")


def copy_rows(src, dst, rows, KS):
    if rows.numel() == 0:
        return
    if not _is_dev(src):
        r = rows.long()
        dst[r] = src[r]
        return
    _lib.check(_lib.lib().oni_copy_rows(_lib.ptr(src), _lib.ptr(dst), _lib.ptr(rows), rows.numel(), KS,
                                        _lib.stream()), "oni_copy_rows")


# ------------------------------------------------------------------------------------------------
# X01 payload packing (csrc/kernels/x01.hip)
# ------------------------------------------------------------------------------------------------
def x01_packed_len(T: int, L: int, H: int, KS: int, tail_len: int) -> int:
    return T * (KS // 4) + L * (KS // 2) + H * KS + tail_len


def x01_pack(dn, tiny, light, heavy, KS: int, tail_off: int, tail_len: int, O8: int, O: int, out) -> None:
    """Tiny rows as four offset bytes per int32 word, light rows as two offset 16-bit halves,
    heavy rows + tail as int32 (csrc/kernels/x01.hip)."""
    T, L, H = tiny.numel(), light.numel(), heavy.numel()
    if not _is_dev(dn):
        q, half = KS // 4, KS // 2
        rows = dn[: tail_off].view(-1, KS)
        nt, nl = T * q, L * half
        if T:
            tv = (rows[tiny.long()].to(torch.int64) + O8).view(T, q, 4)
            out[:nt] = _u32_to_i32(tv[..., 0] | (tv[..., 1] << 8) | (tv[..., 2] << 16) | (tv[..., 3] << 24)).reshape(-1)
        if L:
            lv = (rows[light.long()].to(torch.int64) + O).view(L, half, 2)
            out[nt:nt + nl] = _u32_to_i32(lv[..., 0] | (lv[..., 1] << 16)).reshape(-1)
        out[nt + nl:nt + nl + H * KS] = rows[heavy.long()].reshape(-1)
        out[nt + nl + H * KS:nt + nl + H * KS + tail_len] = dn[tail_off:tail_off + tail_len]
        return
    _lib.check(_lib.lib().oni_x01_pack(_lib.ptr(dn), _lib.ptr(tiny), T, _lib.ptr(light), L, _lib.ptr(heavy), H, KS,
                                       tail_off, tail_len, O8, O, _lib.ptr(out), _lib.stream()), "oni_x01_pack")


def _u32_to_i32(v: torch.Tensor) -> torch.Tensor:
    """int64 tensor of u32 bit patterns → the int32 tensor holding the same bits."""
    return torch.where(v >= 2**31, v - 2**32, v).to(torch.int32)


def x01_unpack(packed, tiny, light, heavy, KS: int, tail_off: int, tail_len: int, WO8: int, WO: int, dn) -> None:
    """Inverse of :func:`x01_pack` after the sum over W ranks (``WO8`` = W·O8, ``WO`` = W·O)."""
    T, L, H = tiny.numel(), light.numel(), heavy.numel()
    if not _is_dev(dn):
        q, half = KS // 4, KS // 2
        nt, nl = T * q, L * half
        rows = dn[: tail_off].view(-1, KS)
        if T:
            v = packed[:nt].to(torch.int64) & 0xFFFFFFFF
            parts = [((v >> (8 * b)) & 0xFF) - WO8 for b in range(4)]
            rows[tiny.long()] = torch.stack(parts, 1).view(T, KS).to(torch.int32)
        if L:
            v = packed[nt:nt + nl].to(torch.int64) & 0xFFFFFFFF
            lo = ((v & 0xFFFF) - WO).to(torch.int32).view(L, half)
            hi = ((v >> 16) - WO).to(torch.int32).view(L, half)
            rows[light.long()] = torch.stack([lo, hi], 2).view(L, KS)
        if H:
            rows[heavy.long()] = packed[nt + nl:nt + nl + H * KS].view(H, KS)
        dn[tail_off:tail_off + tail_len] = packed[nt + nl + H * KS:nt + nl + H * KS + tail_len]
        return
    _lib.check(_lib.lib().oni_x01_unpack(_lib.ptr(packed), _lib.ptr(tiny), T, _lib.ptr(light), L, _lib.ptr(heavy), H,
                                         KS, tail_off, tail_len, WO8, WO, _lib.ptr(dn), _lib.stream()),
               "oni_x01_unpack")


# ------------------------------------------------------------------------------------------------
# scoring / selection
# ------------------------------------------------------------------------------------------------
def score(theta, phi, d1, w1, d2=None, w2=None, tol: float = float("inf"), want_parts=False, hist=None):
    """Event scores (min over the two endpoints when d2/w2 given). Returns (score, s1, s2)."""
    n = d1.numel()
    if not _is_dev(theta):
        sc, s1, s2 = spec.score(theta.numpy(), phi.numpy(), d1.numpy(), w1.numpy(),
                                None if d2 is None else d2.numpy(), None if w2 is None else w2.numpy())
        out = torch.from_numpy(sc)
        if hist is not None:
            sel = sc < tol
            b = spec.f32_key(sc[sel]) >> np.uint32(21)
            hist += torch.from_numpy(np.bincount(b, minlength=2048).astype(np.int32))
        return out, torch.from_numpy(s1), (None if s2 is None else torch.from_numpy(s2))
    KS = theta.shape[-1]
    if phi.shape[-1] != KS:
        raise ValueError("theta/phi row widths differ")
    out = torch.empty(n, dtype=torch.float32, device=theta.device)
    o1 = torch.empty_like(out) if want_parts else None
    o2 = torch.empty_like(out) if (want_parts and d2 is not None) else None
    _lib.check(_lib.lib().oni_score(_lib.ptr(theta), _lib.ptr(phi), KS, _lib.ptr(d1), _lib.ptr(w1),
                                    _lib.ptr(d2), _lib.ptr(w2), n, float(tol), _lib.ptr(out), _lib.ptr(o1),
                                    _lib.ptr(o2), _lib.ptr(hist), _lib.stream()), "oni_score")
    return out, o1, o2


def pair_score(theta, phi, pdoc, pword) -> torch.Tensor:
    """Score of every distinct (doc, word) pair: θ[pdoc]·φ[pword] (K15 SDDMM, k_score dot order)."""
    P = pdoc.numel()
    if not _is_dev(theta):
        return torch.from_numpy(spec.dot_rows(theta.numpy()[pdoc.numpy()], phi.numpy()[pword.numpy()]))
    KS = theta.shape[-1]
    out = torch.empty(P, dtype=torch.float32, device=theta.device)
    _lib.check(_lib.lib().oni_pair_score(_lib.ptr(theta), _lib.ptr(phi), KS, _lib.ptr(pdoc), _lib.ptr(pword), P,
                                         _lib.ptr(out), _lib.stream()), "oni_pair_score")
    return out


def tile_score(theta, phi, item_docs, item_words, item_p0, pair_rc, pdoc, pword) -> torch.Tensor:
    """Pair scores by 16×16 MFMA blocks (K15 MFMA variant, k_tile_score), item-major pair order.

    ``pdoc``/``pword`` (the pairs in the same item-major order) are what the CPU oracle dots; the
    device kernel reads only the item tables. Numerics: k-ordered fmaf chain (spec.dot_rows_fma).
    """
    P = pair_rc.numel()
    if not _is_dev(theta):
        return torch.from_numpy(spec.dot_rows_fma(theta.numpy()[pdoc.numpy()], phi.numpy()[pword.numpy()]))
    KS = theta.shape[-1]
    if phi.shape[-1] != KS:
        raise ValueError("theta/phi row widths differ")
    n_items = item_p0.numel() - 1
    _need(item_docs, torch.int32, "item_docs", n_items * 16)
    _need(item_words, torch.int32, "item_words", n_items * 16)
    _need(item_p0, torch.int64, "item_p0")
    _need(pair_rc, torch.uint8, "pair_rc")
    out = torch.empty(P, dtype=torch.float32, device=theta.device)
    _lib.check(_lib.lib().oni_tile_score(_lib.ptr(theta), _lib.ptr(phi), KS, _lib.ptr(item_docs),
                                         _lib.ptr(item_words), _lib.ptr(item_p0), _lib.ptr(pair_rc), n_items,
                                         _lib.ptr(out), _lib.stream()), "oni_tile_score")
    return out


def event_min(ps, p1, p2=None, tol: float = float("inf"), want_parts=False, hist=None):
    """Per-event score from pair scores: ps[p1] or min(ps[p1], ps[p2]); optional order-key histogram."""
    n = p1.numel()
    if not _is_dev(ps):
        s1 = ps[p1.long()]
        s2 = ps[p2.long()] if p2 is not None else None
        sc = torch.where(s2 < s1, s2, s1) if s2 is not None else s1.clone()
        if hist is not None:
            a = sc.numpy()
            b = spec.f32_key(a[a < tol]) >> np.uint32(21)
            hist += torch.from_numpy(np.bincount(b, minlength=2048).astype(np.int32))
        return sc, (s1 if want_parts else None), (s2 if want_parts else None)
    out = torch.empty(n, dtype=torch.float32, device=ps.device)
    o1 = torch.empty_like(out) if want_parts else None
    o2 = torch.empty_like(out) if (want_parts and p2 is not None) else None
    _lib.check(_lib.lib().oni_event_min(_lib.ptr(ps), _lib.ptr(p1), _lib.ptr(p2), n, float(tol), _lib.ptr(out),
                                        _lib.ptr(o1), _lib.ptr(o2), _lib.ptr(hist), _lib.stream()), "oni_event_min")
    return out, o1, o2


def select_below(score_t: torch.Tensor, tol: float, bmax: int, cap: int):
    """Indices + scores of events with score < tol whose top-11 order-key bucket ≤ bmax (unordered)."""
    if not _is_dev(score_t):
        s = score_t.numpy()
        m = (s < tol) & ((spec.f32_key(s) >> np.uint32(21)) <= bmax)
        idx = np.nonzero(m)[0]
        return torch.from_numpy(idx.astype(np.int64)), torch.from_numpy(s[idx])
    cnt = torch.zeros(1, dtype=torch.int32, device=score_t.device)
    out_i = torch.empty(max(cap, 1), dtype=torch.int64, device=score_t.device)
    out_s = torch.empty(max(cap, 1), dtype=torch.float32, device=score_t.device)
    _lib.check(_lib.lib().oni_select_below(_lib.ptr(score_t), score_t.numel(), float(tol), int(bmax), _lib.ptr(cnt),
                                           _lib.ptr(out_i), _lib.ptr(out_s), cap, _lib.stream()),
               "oni_select_below")
    k = int(cnt.item())
    if k > cap:
        raise RuntimeError(f"select_below overflow: {k} > cap {cap}")
    return out_i[:k], out_s[:k]


def widen_pair(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """[a ‖ b] as non-negative int64 for two int32 tensors holding u32 bits (k_widen_pair: one pass
    instead of cat + int64 conversion + mask)."""
    n = a.numel()
    if b.numel() != n or a.dtype != torch.int32 or b.dtype != torch.int32:
        raise ValueError("widen_pair: two int32 tensors of one length")
    if not _is_dev(a):
        return torch.cat([a, b]).to(torch.int64) & 0xFFFFFFFF
    out = torch.empty(2 * n, dtype=torch.int64, device=a.device)
    _lib.check(_lib.lib().oni_widen_pair(_lib.ptr(a.contiguous()), _lib.ptr(b.contiguous()), n, _lib.ptr(out),
                                         _lib.stream()), "oni_widen_pair")
    return out


def tail_sums(nwk: torch.Tensor, q: torch.Tensor, nk: torch.Tensor, ndk: torch.Tensor, D: int, K: int,
              alpha: float, beta: float, vbeta: float) -> torch.Tensor:
    """Device [8] float64: Σlgamma(n_wk+β), Σlgamma(n_k+Vβ), Σlgamma(n_dk+α), Σlgamma(n_d+Kα) over the
    first ``D`` doc rows, then the health counts (#non-finite q, #negative n_wk/n_k, #negative n_dk)
    -- one pass + a fixed-order reduction (k_tail_partials / k_tail_final), deterministic."""
    V, KS = nwk.shape
    lib = _lib.lib()
    part = torch.empty(lib.oni_tail_grid() * 8, dtype=torch.float64, device=nwk.device)
    out = torch.empty(8, dtype=torch.float64, device=nwk.device)
    _lib.check(lib.oni_tail_sums(_lib.ptr(nwk), _lib.ptr(q), _lib.ptr(nk), _lib.ptr(ndk), V, int(D), int(K), KS,
                                 float(alpha), float(beta), float(vbeta), float(K * alpha), _lib.ptr(part),
                                 _lib.ptr(out), _lib.stream()), "oni_tail_sums")
    return out


def _count_size(t: torch.Tensor) -> int:
    if t.dtype not in (torch.int32, torch.int64):
        raise ValueError("count tables must be int32 or int64")
    return t.element_size()


def theta_rows(n: torch.Tensor, K: int, add: float, den_add: float) -> torch.Tensor:
    """θ = (n + add) / (n_d + den_add) in f32 per row (k_theta_rows), zero past K. ``n`` is an
    int32 count table or the int64 posterior-average sums."""
    D, KS = n.shape
    out = torch.empty(D, KS, dtype=torch.float32, device=n.device)
    _lib.check(_lib.lib().oni_theta_rows(_lib.ptr(n), D, int(K), KS, float(np.float32(add)), float(np.float32(den_add)),
                                         _lib.ptr(out), _count_size(n), _lib.stream()), "oni_theta_rows")
    return out


def phi_rows(nw: torch.Tensor, nk: torch.Tensor, K: int, add: float, vb: float) -> torch.Tensor:
    """φ = (n_wk + add) / (n_k + vb) in f32 (k_phi_rows), zero past K; int32 or int64 counts."""
    V, KS = nw.shape
    out = torch.empty(V, KS, dtype=torch.float32, device=nw.device)
    _lib.check(_lib.lib().oni_phi_rows(_lib.ptr(nw), _lib.ptr(nk), V, int(K), KS, float(np.float32(add)),
                                       float(np.float32(vb)), _lib.ptr(out), _count_size(nw), _count_size(nk),
                                       _lib.stream()),
               "oni_phi_rows")
    return out
