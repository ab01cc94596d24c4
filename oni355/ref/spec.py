"""NumPy specification oracle for every hand-written kernel (tests + the CPU path).

Each function here is the executable spec of one HIP kernel in ``csrc/kernels`` and is written so
that, on identical inputs, it reproduces the kernel **bit-for-bit**: same f32 operation order, no
fused multiply-add (the kernels are built with ``-ffp-contract=off``), same Philox stream.

Behaviour spec sources (the reference has no readable source):
* flow words: SURVEY.md §2.8 (oni-ml FlowWordCreation, [U-M]);
* quantile cuts: SURVEY.md §2.2 C15 (Quantiles.computeDeciles/Quintiles, [U-M]) with the rank
  rule pinned here as ``rank = ceil(num*N/den) - 1`` on the ascending sort;
* scoring: SURVEY.md §2.2 C24 (FlowPostLDA, [U-H]);
* sampler: collapsed Gibbs (replaces oni-lda-c VEM) with the chunked, snapshot
  semantics documented in csrc/kernels/gibbs.hip.
"""
from __future__ import annotations

import numpy as np

U32 = np.uint32
U64 = np.uint64
F32 = np.float32
MASK32 = U64(0xFFFFFFFF)
PAD_WORD = U32(0xFFFFFFFF)

DECILES = [(i, 10) for i in range(1, 10)]
QUINTILES = [(i, 5) for i in range(1, 5)]

PORT_111111 = 65536
PORT_333333 = 65537


# ------------------------------------------------------------------------------------------------
# Philox4x32-10
# ------------------------------------------------------------------------------------------------
def philox10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(x, dtype=U32) for x in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0, c1, c2, c3 = (x.copy() for x in (c0, c1, c2, c3))
    k0 = U32(k0)
    k1 = U32(k1)
    for _ in range(10):
        p0 = c0.astype(U64) * U64(0xD2511F53)
        p1 = c2.astype(U64) * U64(0xCD9E8D57)
        hi0, lo0 = (p0 >> U64(32)).astype(U32), (p0 & MASK32).astype(U32)
        hi1, lo1 = (p1 >> U64(32)).astype(U32), (p1 & MASK32).astype(U32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = U32((int(k0) + 0x9E3779B9) & 0xFFFFFFFF)
        k1 = U32((int(k1) + 0xBB67AE85) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def philox2x32_10(c0, c1, k):
    """Philox2x32-10 (multiplier 0xD256D193, key bump 0x9E3779B9): half the work of the 4x32
    generator where a draw needs two words (the MH sampler's extra doc moves)."""
    c0 = np.asarray(c0, dtype=U32).copy()
    c1 = np.asarray(c1, dtype=U32).copy()
    c0, c1 = np.broadcast_arrays(c0, c1)
    c0, c1 = c0.copy(), c1.copy()
    k = int(k) & 0xFFFFFFFF
    for _ in range(10):
        p = c0.astype(U64) * U64(0xD256D193)
        hi, lo = (p >> U64(32)).astype(U32), (p & MASK32).astype(U32)
        c0, c1 = hi ^ U32(k) ^ c1, lo
        k = (k + 0x9E3779B9) & 0xFFFFFFFF
    return c0, c1


def mh_move_key(sweep, move, seed0, seed1):
    """Per-sweep key of the Philox2x32 stream of MH doc move ``move`` ≥ 1 (counter = (pos, doc
    key)); one Philox4x32 block of (sweep, 2 + move, 'MH', 0) under the run seed."""
    return int(philox10(U32(sweep), U32(2 + move), U32(0x4D48), U32(0), seed0, seed1)[0])


def token_rand(pos, key, sweep, stream, seed0, seed1):
    """The u32 draw of token (doc key, pos) in (sweep, stream): mirrors the kernel's pick4."""
    pos = np.asarray(pos, dtype=U32)
    r = philox10(pos >> U32(2), key, U32(sweep), U32(stream), seed0, seed1)
    sel = pos & U32(3)
    return np.select([sel == 0, sel == 1, sel == 2], [r[0], r[1], r[2]], r[3]).astype(U32)


def mix32(x):
    """lowbias32 integer mixer (oni_common.h mix32): the seed-free initial topic of a word."""
    x = np.asarray(x, dtype=U64) & MASK32
    x ^= x >> U64(16)
    x = (x * U64(0x7FEB352D)) & MASK32
    x ^= x >> U64(15)
    x = (x * U64(0x846CA68B)) & MASK32
    x ^= x >> U64(16)
    return x.astype(U32)


def u01(r):
    return (np.asarray(r, dtype=U32) >> U32(8)).astype(F32) * F32(5.9604644775390625e-08)


def split_seed(seed: int) -> tuple[int, int]:
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF


# ------------------------------------------------------------------------------------------------
# keys / quantiles / bins (K01, K02)
# ------------------------------------------------------------------------------------------------
def f32_key(x):
    u = np.asarray(x, dtype=F32).view(U32)
    neg = (u & U32(0x80000000)) != 0
    return np.where(neg, ~u, u | U32(0x80000000)).astype(U32)


def key_f32(k):
    k = np.asarray(k, dtype=U32)
    neg = (k & U32(0x80000000)) == 0
    return np.where(neg, ~k, k & U32(0x7FFFFFFF)).astype(U32).view(F32)


def i64_keys(x):
    x = np.asarray(x, dtype=np.int64)
    return np.clip(x, 0, 0xFFFFFFFF).astype(U32)


def quantile_ranks(n: int, fracs) -> np.ndarray:
    """0-based ascending ranks of the cut points: ceil(num*n/den) - 1 (clamped to [0, n-1])."""
    r = np.array([(num * n + den - 1) // den - 1 for num, den in fracs], dtype=np.int64)
    return np.clip(r, 0, max(n - 1, 0))


def quantile_cuts(keys, fracs) -> np.ndarray:
    keys = np.asarray(keys, dtype=U32)
    if keys.size == 0:
        return np.zeros(len(fracs), dtype=U32)
    ranks = quantile_ranks(keys.size, fracs)
    part = np.partition(keys, np.unique(ranks))
    return part[ranks].astype(U32)


def radix_hist(keys, shift: int, nbits: int, prefixes, mask: int) -> np.ndarray:
    """k_radix_hist: per live prefix, histogram of digit (key >> shift) & (2^nbits-1)."""
    keys = np.asarray(keys, dtype=U32)
    B = 1 << nbits
    hi = keys & U32(mask)
    digit = ((keys >> U32(shift)) & U32(B - 1)).astype(np.int64)
    out = np.zeros((len(prefixes), B), dtype=np.int64)
    for i, p in enumerate(prefixes):
        out[i] = np.bincount(digit[hi == U32(p)], minlength=B)
    return out


def bin_keys(keys, cuts):
    keys = np.asarray(keys, dtype=U32)
    cuts = np.asarray(cuts, dtype=U32)
    return (keys[:, None] > cuts[None, :]).sum(axis=1).astype(np.uint8)


# ------------------------------------------------------------------------------------------------
# flow word creation (K03)
# ------------------------------------------------------------------------------------------------
def flow_time(hour, minute, second):
    h = np.asarray(hour).astype(F32)
    m = np.asarray(minute).astype(F32)
    s = np.asarray(second).astype(F32)
    return (h + m / F32(60.0)) + s / F32(3600.0)


def flow_keys(hour, minute, second, ibyt, ipkt):
    return f32_key(flow_time(hour, minute, second)), i64_keys(ibyt), i64_keys(ipkt)


def flow_port_rule(sport, dport):
    """Returns (port_code, src_dir, dst_dir) per SURVEY.md §2.8 table (first matching row wins)."""
    sp = np.asarray(sport, dtype=np.int64)
    dp = np.asarray(dport, dtype=np.int64)
    conds = [
        (sp == 0) & (dp == 0),
        (dp == 0) & (sp > 0),
        (sp == 0) & (dp > 0),
        (sp <= 1024) & (dp <= 1024),
        (sp <= 1024) & (dp > 1024),
        (sp > 1024) & (dp <= 1024),
    ]
    port = np.select(conds, [0, sp, dp, PORT_111111, sp, dp], PORT_333333).astype(np.int64)
    sdir = np.select(conds, [0, 1, 0, 0, 1, 0], 0).astype(np.int64)
    ddir = np.select(conds, [0, 0, 1, 0, 0, 1], 0).astype(np.int64)
    return port, sdir, ddir


def flow_wordify(sport, dport, tkey, bkey, pkey, tcuts, bcuts, pcuts):
    tb = bin_keys(tkey, tcuts).astype(np.int64)
    bb = bin_keys(bkey, bcuts).astype(np.int64)
    pb = bin_keys(pkey, pcuts).astype(np.int64)
    port, sdir, ddir = flow_port_rule(sport, dport)
    base = (port << 11) | (tb << 7) | (bb << 3) | pb
    return (base | (sdir << 28)).astype(U32), (base | (ddir << 28)).astype(U32)


def flow_word_fields(word):
    w = np.asarray(word, dtype=np.int64)
    return (w >> 28) & 1, (w >> 11) & 0x1FFFF, (w >> 7) & 0xF, (w >> 3) & 0xF, w & 0x7


def flow_word_str(word: int) -> str:
    w = int(word)
    d, port, tb, bb, pb = (w >> 28) & 1, (w >> 11) & 0x1FFFF, (w >> 7) & 0xF, (w >> 3) & 0xF, w & 0x7
    p = {PORT_111111: "111111", PORT_333333: "333333"}.get(port, str(port))
    return f"{'-1_' if d else ''}{p}_{tb}_{bb}_{pb}"


def flow_word_from_str(s: str) -> int:
    d = s.startswith("-1_")
    if d:
        s = s[3:]
    p, tb, bb, pb = s.split("_")
    port = {"111111": PORT_111111, "333333": PORT_333333}.get(p, None)
    port = int(p) if port is None else port
    return (int(d) << 28) | (port << 11) | (int(tb) << 7) | (int(bb) << 3) | int(pb)


# ------------------------------------------------------------------------------------------------
# SELL fill (K09 second half)
# ------------------------------------------------------------------------------------------------
def sell_fill(chunk_doc, chunk_pos0, chunk_len, S, slice_off, doc_pair_ptr, pair_tokoff, pair_word, pair_cnt,
              tok_word):
    chunk_doc = np.asarray(chunk_doc)
    for i in np.nonzero(chunk_doc >= 0)[0]:
        d = int(chunk_doc[i])
        lo, hi = int(doc_pair_ptr[d]), int(doc_pair_ptr[d + 1])
        off = int(slice_off[i // S]) + i % S
        pos0, ln = int(chunk_pos0[i]), int(chunk_len[i])
        # expand this doc's pairs into token words, then take [pos0, pos0+len)
        words = np.repeat(np.asarray(pair_word[lo:hi]), np.asarray(pair_cnt[lo:hi]))
        tok_word[off + np.arange(ln) * S] = words[pos0:pos0 + ln].astype(U32)
    return tok_word


# ------------------------------------------------------------------------------------------------
# collapsed Gibbs: init / sweep / apply (K10-K12)
# ------------------------------------------------------------------------------------------------
def _chunk_geometry(st, S):
    n_slices = st["slice_len"].shape[0]
    C = n_slices * S
    cid = np.arange(C)
    return cid // S, cid % S


def fma_f32(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """Correctly rounded f32 fma(a, b, c) (= v_fma_f32), emulated exactly in float64.

    a·b is exact in f64 (24+24 bits); s = a·b + c is rounded once, its error e is recovered with
    TwoSum. round_f32(s) is then the right answer unless s sits exactly on a midpoint between two
    f32 values with e ≠ 0, in which case e decides the direction.
    """
    p = a.astype(np.float64) * b.astype(np.float64)
    c64 = c.astype(np.float64)
    s = p + c64
    bb = s - p
    e = (p - (s - bb)) + (c64 - bb)
    r = s.astype(F32)
    r64 = r.astype(np.float64)
    other = np.nextafter(r, np.where(s > r64, np.inf, -np.inf).astype(F32))
    mid = (s != r64) & ((r64 + other.astype(np.float64)) * 0.5 == s) & (e != 0)
    if mid.any():
        # exact value = s + e: above the midpoint -> the larger neighbour of s, else the smaller
        hi = np.where(r64 > s, r, other)
        lo = np.where(r64 > s, other, r)
        r = np.where(mid, np.where(e > 0, hi, lo), r)
    return r.astype(F32)


def gibbs_qfix(nk_next: np.ndarray, K: int, vbeta: float) -> np.ndarray:
    """Per-topic constants of the token exclusion on the word side (k_apply writes them with q).

    With D_k = n_k + Vβ (the sweep-start denominator of q) the word factor of a token's own topic
    with the token removed is (n_wk − 1 + β)/(D_k − 1) = q_wk·A_k − B_k, A_k = D_k/(D_k − 1),
    B_k = 1/(D_k − 1). Returned as [2, KS] f32 (row 0 = A, row 1 = B); topics with n_k = 0 (never a
    token's own topic) get A = 1, B = 0."""
    KS = nk_next.shape[0]
    out = np.zeros((2, KS), dtype=F32)
    out[0] = F32(1)
    den = nk_next.astype(F32) + F32(vbeta)
    dm1 = den - F32(1)
    ok = (np.arange(KS) < K) & (nk_next >= 1)
    out[0, ok] = (den[ok] / dm1[ok]).astype(F32)
    out[1, ok] = (F32(1) / dm1[ok]).astype(F32)
    return out


def excluded_q(qz: np.ndarray, zo: np.ndarray, qfix: np.ndarray) -> np.ndarray:
    """q'_{w,zo} = fma(q_{w,zo}, A_zo, −B_zo): the word factor of the token's own topic without
    the token (the sweep-start snapshot counts every token at its sweep-start topic)."""
    return fma_f32(qz.astype(F32), qfix[0][zo], -qfix[1][zo])


def gibbs_pass(st: dict, G: int, KP: int, K: int, alpha: float, seed0: int, seed1: int, init: bool,
               sweep: int, chunk_len: np.ndarray, word_init: bool = False):
    """One init (init=True) or sweep pass over numpy state arrays, in place.

    A sweep draws every token from the collapsed conditional with the token removed from BOTH
    sides (SURVEY.md §2.6 K10 "remove its old z"):

        p_k ∝ (n_dk^¬t + α) · (n_wk^¬t + β)/(n_k^¬t + Vβ)

    The doc side n_dk is exact within a chunk (sequential updates); the word side is the
    sweep-start snapshot q (AD-LDA staleness), which counts the token itself at its sweep-start
    topic zo, so the factor of topic zo is replaced by q' = fma(q_zo, A_zo, −B_zo)
    (:func:`excluded_q`, st["qfix"] from :func:`gibbs_qfix`). Weight numerics (the kernels replay
    them bit for bit):

    * G = 1 (k_gibbs_x1 / k_gibbs): P_j = fma(a_j, q_j, P_{j−1}) with q_zo := q', a_j = n_j + α.
    * G > 1 (k_gibbs_ldsg / k_gibbs): lane g chains its KP topics, P_j = fma(e_j, q_j, P_{j−1}) with
      e_j = a_j except e_zo = a_zo · f, f = q' / q_zo (the LDS row of the owning lane is scaled for
      the one step, the q row stays in registers); lanes are combined by a Hillis-Steele scan.

    The draw is the first topic whose running weight exceeds u·total (count of P_j ≤ thr, capped
    at K − 1).

    Lagged word side (``st["tok_zlag"]`` present, ONI_X01_LAG, models/gibbs.py): q and qfix come
    from the global counts one sweep older than the doc rows, which count every token at its topic
    of that older sweep, ``zl = tok_zlag`` -- so the word-side exclusion (q' in place of q, or the
    row scale f) is taken at zl while the doc side still removes the token at zo; the pass then
    writes tok_zlag := zo (the topics the next sweep's word side will count).

    st keys: tok_word u32, tok_z u8, slice_off i64, slice_len i32, chunk_doc i32, chunk_pos0 i32,
    chunk_key u32, chunk_multi u8, ndk_src i32 [D,KS], ndk_dst i32 [D,KS], q f32 [V,KS],
    qfix f32 [2,KS] (sweeps), dnwk i32 [V,KS], dnk i32 [KS].
    """
    S = 64 // G
    KS = G * KP
    slc, lane = _chunk_geometry(st, S)
    doc = st["chunk_doc"]
    live = doc >= 0
    C = doc.shape[0]
    n = np.zeros((C, KS), dtype=np.int32)
    if not init:
        n[live] = st["ndk_src"][doc[live]]
        qfix = st["qfix"]
    lag = not init and st.get("tok_zlag") is not None
    n_start = n.copy()
    clen = np.where(live, chunk_len, 0)
    alpha32 = F32(alpha)
    stream = 0 if init else 1
    sw = 0 if init else sweep
    for s in range(int(clen.max(initial=0))):
        act = np.nonzero(clen > s)[0]
        A = act.size
        ar = np.arange(A)
        idx = st["slice_off"][slc[act]] + s * S + lane[act]
        w = st["tok_word"][idx].astype(np.int64)
        pos = st["chunk_pos0"][act].astype(U32) + U32(s)
        rr = token_rand(pos, st["chunk_key"][act], sw, stream, seed0, seed1)
        if init:
            if word_init:  # seed-free start: every token of a word in the word's hashed topic
                rr = mix32(w)
            z = ((rr.astype(U64) * U64(K)) >> U64(32)).astype(np.int64)
            n[act, z] += 1
            st["tok_z"][idx] = z.astype(np.uint8)
            np.add.at(st["dnwk"], (w, z), 1)
            continue
        zo = st["tok_z"][idx].astype(np.int64)
        zl = st["tok_zlag"][idx].astype(np.int64) if lag else zo
        n[act, zo] -= 1
        qv = st["q"][w].copy()
        qz = qv[ar, zl]
        qe = excluded_q(qz, zl, qfix)
        av = n[act].astype(F32) + alpha32
        if G == 1:
            qv[ar, zl] = qe
        else:
            f = (qe / qz).astype(F32)
            av[ar, zl] = (av[ar, zl] * f).astype(F32)
        avg = av.reshape(-1, G, KP)
        qg = qv.reshape(-1, G, KP)
        loc = np.empty_like(avg)
        run = np.zeros(avg.shape[:2], dtype=F32)
        for j in range(KP):
            run = fma_f32(avg[:, :, j], qg[:, :, j], run)
            loc[:, :, j] = run
        if G == 1:
            cum = loc.reshape(-1, KS)
            total = cum[:, -1]
        else:
            incl = loc[:, :, -1].copy()
            d = 1
            while d < G:
                prev = incl.copy()
                incl[:, d:] = prev[:, d:] + prev[:, :-d]
                d <<= 1
            excl = np.zeros_like(incl)
            excl[:, 1:] = incl[:, :-1]
            cum = (excl[:, :, None] + loc).reshape(-1, KS)
            total = incl[:, -1]
        thr = u01(rr) * total
        cnt = (cum <= thr[:, None]).sum(axis=1)
        zn = np.minimum(cnt, K - 1).astype(np.int64)
        n[act, zn] += 1
        ch = zn != zo
        if lag:
            st["tok_zlag"][idx] = zo.astype(np.uint8)
        st["tok_z"][idx[ch]] = zn[ch].astype(np.uint8)
        np.add.at(st["dnwk"], (w[ch], zo[ch]), -1)
        np.add.at(st["dnwk"], (w[ch], zn[ch]), 1)
    d = n - n_start
    multi = live & (st["chunk_multi"] != 0)
    single = live & ~multi
    st["ndk_dst"][doc[single]] = n[single]
    np.add.at(st["ndk_dst"], doc[multi], d[multi])
    st["dnk"] += d[live].sum(axis=0).astype(np.int32)


def gibbs_apply(nwk, dcur, dnk_cur, nk_cur, K, beta, vbeta):
    """Returns (nwk', nk', q, qfix) exactly as k_apply computes them."""
    nwk = nwk + dcur
    nk = nk_cur + dnk_cur
    den = nk.astype(F32) + F32(vbeta)
    q = (nwk.astype(F32) + F32(beta)) / den[None, :]
    q[:, K:] = 0
    return nwk, nk, q.astype(F32), gibbs_qfix(nk, K, vbeta)


# ------------------------------------------------------------------------------------------------
# Metropolis-Hastings sampler with sweep-static alias proposals (k_mh_alias / k_gibbs_mh)
# ------------------------------------------------------------------------------------------------
MH_BIAS = 128     # multi-chunk docs keep n_view - n_src + MH_BIAS in the kernel's u8 LDS cells
MH_MAX_CHUNK = 127


def alias_table(wts: np.ndarray):
    """Vose alias tables of the rows of ``wts`` ([R, K] f32, positive), exactly as k_mh_alias builds
    them (one lane per row, sequential f32): tot = Σ_k w_k in order, p_k = w_k · (K / tot); indices
    with p < 1 are pushed on the small stack, the others on the large one (both in k order); then
    while both are non-empty: s = pop small, l = pop large, bucket s := (p_s, alias l),
    p_l := (p_l + p_s) − 1, l pushed back on small if p_l < 1 else on large. Buckets left over
    keep their own index. Entry = thr24 << 8 | alias with thr24 = min(⌊p · 2^24⌋, 2^24 − 1)
    (2^24 − 1 and alias = itself for p ≥ 1): a draw takes j = ⌊r·K / 2^32⌋ and keeps j when the
    low word's top 24 bits are below thr24, else its alias (:func:`alias_draw`).
    Returns (tables [R, K] u32, tot [R] f32)."""
    wts = np.ascontiguousarray(wts, dtype=F32)
    R, K = wts.shape
    tot = np.zeros(R, dtype=F32)
    for k in range(K):
        tot = (tot + wts[:, k]).astype(F32)
    scale = (F32(K) / tot).astype(F32)
    p = (wts * scale[:, None]).astype(F32)
    stk = np.zeros((R, K), dtype=np.int64)
    ns = np.zeros(R, dtype=np.int64)
    nl = np.zeros(R, dtype=np.int64)
    rows = np.arange(R)
    for k in range(K):
        sm = p[:, k] < F32(1)
        stk[rows[sm], ns[sm]] = k
        stk[rows[~sm], K - 1 - nl[~sm]] = k
        ns += sm
        nl += ~sm
    prob = np.ones((R, K), dtype=F32)
    alias = np.tile(np.arange(K, dtype=np.int64), (R, 1))
    for _ in range(K):
        r = np.nonzero((ns > 0) & (nl > 0))[0]
        if r.size == 0:
            break
        s_ = stk[r, ns[r] - 1]
        ns[r] -= 1
        l_ = stk[r, K - nl[r]]
        nl[r] -= 1
        prob[r, s_] = p[r, s_]
        alias[r, s_] = l_
        pl = ((p[r, l_] + p[r, s_]).astype(F32) - F32(1)).astype(F32)
        p[r, l_] = pl
        sm = pl < F32(1)
        stk[r[sm], ns[r[sm]]] = l_[sm]
        ns[r[sm]] += 1
        stk[r[~sm], K - 1 - nl[r[~sm]]] = l_[~sm]
        nl[r[~sm]] += 1
    full = prob >= F32(1)
    thr = np.minimum((prob * F32(16777216.0)).astype(np.int64), 0xFFFFFF)
    thr = np.where(full, 0xFFFFFF, thr)
    alias = np.where(full, np.arange(K)[None, :], alias)
    return ((thr << 8) | alias).astype(U32), tot


def alias_draw(tab_rows: np.ndarray, r: np.ndarray, K: int) -> np.ndarray:
    """Topic drawn from alias rows ``tab_rows`` ([A, K] u32) with u32 randoms ``r`` ([A])."""
    prod = np.asarray(r, dtype=U32).astype(U64) * U64(K)
    j = (prod >> U64(32)).astype(np.int64)
    coin = ((prod & MASK32) >> U64(8)).astype(np.int64)
    e = tab_rows[np.arange(j.size), j].astype(np.int64)
    return np.where(coin < (e >> 8), j, e & 0xFF)


MH_CDF_BUCKETS = 16  # level-1 entries per word (one 64-B row)


def mh_bucket_width(K: int) -> int:
    """Topics per level-1 bucket of the word proposal: 8 up to K = 128, 16 above (≤ 16 buckets)."""
    return 8 if K <= 128 else 16


def word_cdf(q: np.ndarray, K: int) -> np.ndarray:
    """Level-1 table of the word proposal ∝ q[w, ·] (k_mh_cdf): topics in buckets of
    :func:`mh_bucket_width` consecutive topics; S_b = Σ_k q_k over the bucket (sequential f32 in k),
    C[b] = Σ_{b' ≤ b} S_b' (sequential f32), entries past the last bucket repeat the total.
    Returns [V, 16] f32; C[:, 15] is the proposal's normaliser Z."""
    q = np.asarray(q, dtype=F32)
    V = q.shape[0]
    Wb = mh_bucket_width(K)
    nb = (K + Wb - 1) // Wb
    C = np.zeros((V, MH_CDF_BUCKETS), dtype=F32)
    c = np.zeros(V, dtype=F32)
    for b in range(MH_CDF_BUCKETS):
        if b < nb:
            sb = np.zeros(V, dtype=F32)
            for j in range(Wb):
                k = b * Wb + j
                if k < K:
                    sb = (sb + q[:, k]).astype(F32)
            c = (c + sb).astype(F32)
        C[:, b] = c
    return C


def word_cdf_draw(C: np.ndarray, qrow: np.ndarray, r: np.ndarray, K: int) -> np.ndarray:
    """Topic of the word proposal (inverse CDF, two levels): y = u(r)·Z; bucket b = #{i : C[i] ≤ y}
    (capped at the last bucket); y' = y − C[b − 1] (C[−1] = 0); inside the bucket the running f32
    sum of q from 0, topic = b·W + #{j : cum_j ≤ y'} capped at the bucket's last topic."""
    A = C.shape[0]
    ar = np.arange(A)
    Wb = mh_bucket_width(K)
    nb = (K + Wb - 1) // Wb
    y = (u01(r) * C[:, MH_CDF_BUCKETS - 1]).astype(F32)
    b = np.minimum((C <= y[:, None]).sum(axis=1), nb - 1)
    base = np.where(b > 0, C[ar, np.maximum(b - 1, 0)], F32(0)).astype(F32)
    y2 = (y - base).astype(F32)
    cum = np.zeros(A, dtype=F32)
    cnt = np.zeros(A, dtype=np.int64)
    for j in range(Wb):
        k = b * Wb + j
        ok = k < K
        cum = (cum + np.where(ok, qrow[ar, np.minimum(k, K - 1)], F32(0))).astype(F32)
        cnt += (ok & (cum <= y2)).astype(np.int64)
    last = np.minimum(Wb, K - b * Wb) - 1
    return b * Wb + np.minimum(cnt, last)


def mh_tables(q: np.ndarray, nk: np.ndarray, ndk_src: np.ndarray, long_rows: np.ndarray, K: int, alpha: float,
              vbeta: float, word: str = "alias"):
    """Per-sweep tables of the MH sampler (k_mh_alias / k_mh_cdf): the word proposal ∝ q[w, k]
    (sweep-start word factor), the doc proposal ∝ n_dk + α (sweep-start row) of every document over
    several chunks as alias rows, and g_k = 1/(n_k + Vβ + 1) (the word factor a token adds to a
    topic it moves into). ``word`` "alias": every word's alias row as records {entry, q_j,
    q_alias(j), Σ_k q_k} (the kernel's 16-B gather; small vocabularies); "cdf": every word's
    level-1 CDF row (:func:`word_cdf`; the second level is the q row itself; large ones).
    Returns (wtab, wsum, dalias [n_long, K] u32, g [KS] f32) with wtab = walias [V, K, 4] u32 and
    wsum [V] f32, or wtab = wcdf [V, 16] f32 and wsum None."""
    if word == "cdf":
        wtab, wsum = word_cdf(q[:, :K], K), None
    else:
        ent, wsum = alias_table(q[:, :K])
        q32 = np.ascontiguousarray(q[:, :K], dtype=F32)
        al = (ent & U32(0xFF)).astype(np.int64)
        wtab = np.stack([ent, q32.view(U32), np.take_along_axis(q32, al, axis=1).view(U32),
                         np.repeat(wsum[:, None], K, axis=1).astype(F32).view(U32)], axis=2).astype(U32)
    b = ndk_src[np.asarray(long_rows, dtype=np.int64), :K].astype(F32) + F32(alpha)
    dalias = alias_table(b)[0] if b.shape[0] else np.zeros((0, K), dtype=U32)
    g = (F32(1) / ((nk.astype(F32) + F32(vbeta)).astype(F32) + F32(1))).astype(F32)
    return wtab, wsum, dalias, g


def mh_moves(nn, bb, qrow, zo, qe, multi, Nd, s, zslice, drows, wtab, wsum, g, pos, key, sweep, seed0, seed1,
             K, alpha, doc_moves=1):
    """The MH moves of one token per row (see :func:`gibbs_pass_mh`). ``nn`` doc counts without the
    token (the chunk's view), ``bb`` sweep-start doc rows (with the token), ``qrow`` sweep-start q
    rows (with the token), ``qe`` the word factor of ``zo`` without it, ``Nd`` other tokens in the
    chunk, ``s`` the token's position, ``zslice`` current topics of the chunk's positions,
    ``drows`` alias rows of the doc (multi-chunk docs), ``wtab`` / ``wsum`` the word's alias rows
    [A, K] u32 and row sums, or (``wsum`` None) its level-1 CDF rows [A, 16] f32 (:func:`word_cdf`,
    Z = wtab[:, 15]), ``g`` [KS] = 1/(D + 1). Returns the new topics."""
    A = zo.shape[0]
    ar = np.arange(A)
    a32 = F32(alpha)
    kalpha = (F32(K) * a32).astype(F32)
    inv_a = F32(1.0 / alpha)
    one = F32(1)
    Ndf = np.asarray(Nd).astype(F32)
    tot = (Ndf + kalpha).astype(F32)

    def aw(k):
        return (nn[ar, k].astype(F32) + a32).astype(F32)

    def qx(k):  # q' (word factor without the token)
        return np.where(k == zo, qe, qrow[ar, k]).astype(F32)

    def bn(k):  # sweep-start doc row without the token, + α
        return ((bb[ar, k] - (k == zo)).astype(F32) + a32).astype(F32)
    # word move (from zo; proposal = the word's CDF over the snapshot q, which holds the token at zo)
    r0, r1, r2, r3 = philox10(pos, key, U32(sweep), U32(2), seed0, seed1)
    if wsum is None:
        t = word_cdf_draw(wtab, qrow, r0, K)
        wsum = wtab[:, MH_CDF_BUCKETS - 1]
    else:
        t = alias_draw(wtab, r0, K)
    d = (qrow[ar, zo] - qe).astype(F32)
    zt = ((wsum - d).astype(F32) + ((one - qrow[ar, t]).astype(F32) * g[t]).astype(F32)).astype(F32)
    num = (aw(t) * wsum).astype(F32)
    den = (aw(zo) * zt).astype(F32)
    acc = (t != zo) & ((u01(r1) * den).astype(F32) < num)
    sc = np.where(acc, t, zo)
    for c in range(doc_moves):
        if c:
            r2, r3 = philox2x32_10(pos, key, mh_move_key(sweep, c, seed0, seed1))
        y = (u01(r2) * tot).astype(F32)
        pick = y < Ndf
        pp = y.astype(np.int64)
        pp = np.where(pp >= s, pp + 1, pp)
        tz = zslice[ar, np.where(pick, pp, 0)]
        tu = np.minimum(((y - Ndf).astype(F32) * inv_a).astype(F32).astype(np.int64), K - 1)
        t = np.where(pick, tz, tu)
        if drows is not None and multi.any():
            t = np.where(multi, alias_draw(drows, r2, K), t)
        qt, qs = qx(t), qx(sc)
        u = u01(r3)
        num = np.where(multi, ((aw(t) * qt).astype(F32) * bn(sc)).astype(F32), qt)
        den = np.where(multi, ((aw(sc) * qs).astype(F32) * bn(t)).astype(F32), qs)
        ok = (u * den).astype(F32) < num
        # a multi-chunk doc's table holds the token at zo; from sc ≠ zo a draw of zo stands for
        # sc with probability 1/(b_zo + α) (a no-op), so zo is proposed with (b_zo^¬ + α)/N
        sw = multi & (t == zo) & (sc != zo)
        bz = (bb[ar, zo].astype(F32) + a32).astype(F32)
        wn = bn(zo)
        ok_sw = ((u * bz).astype(F32) < wn) & (((u * den).astype(F32) * bz).astype(F32) < (num * wn).astype(F32))
        ok = np.where(sw, ok_sw, ok) & (t != sc)
        sc = np.where(ok, t, sc)
    return sc


def gibbs_pass_mh(st: dict, KS: int, K: int, alpha: float, seed0: int, seed1: int, sweep: int,
                  chunk_len: np.ndarray, doc_moves: int = 1):
    """One Metropolis-Hastings sweep (k_gibbs_mh), in place; one-lane units (S = 64 chunks a slice).

    Target per token (zo = its topic, counts without it, AD-LDA word side as in :func:`gibbs_pass`):
        π(k) ∝ (n_dk^¬ + α) · q'_k,   q'_k = q[w, k] (k ≠ zo), q'_zo = fma(q_zo, A_zo, −B_zo).
    π does not depend on zo, but the sweep's proposal tables do (they count the token at zo). Every
    move is therefore an MH step with the proposal the tables WOULD give with the token at the
    current state x -- a kernel reversible w.r.t. π, so their composition leaves π invariant
    (tests/test_mh_conditional.py). Philox blocks (pos, doc key, sweep, 2 + c) → r0..r3:

    * word move, from zo only (r0 proposes t ∝ q[w, ·] -- from the word's alias row, or by the
      two-level inverse CDF :func:`word_cdf_draw`: level 1 the per-sweep bucket sums, level 2 the q
      row itself -- r1 accepts): ratio (n_t^¬+α)·Z_zo / ((n_zo^¬+α)·Z_t) with Z_zo = the proposal's
      total (alias row sum / CDF total) and
      Z_t = (Z_zo − (q_zo − q'_zo)) + (1 − q_t)·g_t, the sum the table would have with the token
      at t (g_t = 1/(D_t + 1)).
    * ``doc_moves`` doc moves (r2 proposes, r3 accepts; move c > 0 draws (r2, r3) from
      Philox2x32-10 on (pos, doc key) under the per-sweep key :func:`mh_move_key`). One-chunk
      documents propose ∝ n_dk^¬ + α -- with y = u(r2)·(L − 1 + Kα), y < L − 1 picks the current
      topic of another token of the chunk (position ⌊y⌋, skipping its own), else topic
      ⌊(y − (L − 1))/α⌋ -- a state-free proposal: ratio q'_t / q'_x. Documents over several chunks
      propose from the alias table of their sweep-start row b + α: ratio
      (n_t^¬+α)·q'_t·(b_x^¬+α) / ((n_x^¬+α)·q'_x·(b_t^¬+α)), b^¬ = b without the token; a draw of
      zo from x ≠ zo is kept with probability (b_zo^¬ + α)/(b_zo + α) first.

    A move is taken when u(r)·den < num (f32). st as for :func:`gibbs_pass` plus the word proposal
    (``walias`` [V, K, 4] u32 records and ``wsum`` [V] f32, or ``wcdf`` [V, 16] f32 level-1 CDF
    rows), ``dalias`` [n_long, K] u32, ``mh_g`` [KS] f32 (:func:`mh_tables`)
    and ``chunk_dslot`` [C] i32 (row of dalias of a multi-chunk doc's chunk, −1 otherwise)."""
    S = 64
    slc, lane = _chunk_geometry(st, S)
    doc = st["chunk_doc"]
    live = doc >= 0
    C = doc.shape[0]
    n = np.zeros((C, KS), dtype=np.int32)
    n[live] = st["ndk_src"][doc[live]]
    b = n.copy()
    n_start = n.copy()
    multi_c = live & (st["chunk_multi"] != 0)
    clen = np.where(live, chunk_len, 0).astype(np.int64)
    if clen.max(initial=0) > MH_MAX_CHUNK:
        raise ValueError("the MH sampler needs chunks of at most 127 tokens")
    qfix = st["qfix"]
    dalias = st["dalias"]
    cdf = st.get("wcdf") is not None
    dslot = st["chunk_dslot"].astype(np.int64)
    base = st["slice_off"][slc].astype(np.int64) + lane
    for s in range(int(clen.max(initial=0))):
        act = np.nonzero(clen > s)[0]
        ar = np.arange(act.size)
        idx = base[act] + s * S
        w = st["tok_word"][idx].astype(np.int64)
        zo = st["tok_z"][idx].astype(np.int64)
        pos = st["chunk_pos0"][act].astype(U32) + U32(s)
        n[act, zo] -= 1
        qrow = st["q"][w]
        qe = excluded_q(qrow[ar, zo], zo, qfix)
        zp = np.minimum(np.arange(int(clen[act].max()))[None, :], clen[act][:, None] - 1)
        zslice = st["tok_z"][base[act][:, None] + zp * S].astype(np.int64)
        zn = mh_moves(n[act], b[act], qrow, zo, qe, multi_c[act], clen[act] - 1, s, zslice,
                      dalias[np.where(multi_c[act], dslot[act], 0)] if dalias.shape[0] else None,
                      st["wcdf"][w] if cdf else st["walias"][w, :, 0], None if cdf else st["wsum"][w],
                      st["mh_g"], pos, st["chunk_key"][act], sweep, seed0, seed1, K, alpha,
                      doc_moves)
        n[act, zn] += 1
        ch = zn != zo
        st["tok_z"][idx[ch]] = zn[ch].astype(np.uint8)
        np.add.at(st["dnwk"], (w[ch], zo[ch]), -1)
        np.add.at(st["dnwk"], (w[ch], zn[ch]), 1)
    d = n - n_start
    single = live & ~multi_c
    st["ndk_dst"][doc[single]] = n[single]
    np.add.at(st["ndk_dst"], doc[multi_c], d[multi_c])
    st["dnk"] += d[live].sum(axis=0).astype(np.int32)


# ------------------------------------------------------------------------------------------------
# scoring (K15)
# ------------------------------------------------------------------------------------------------
def dot_rows(theta_rows, phi_rows):
    s = np.zeros(theta_rows.shape[0], dtype=F32)
    for k in range(theta_rows.shape[1]):
        s = s + theta_rows[:, k] * phi_rows[:, k]
    return s


def dot_rows_fma(theta_rows, phi_rows):
    """k-ordered fmaf chain from 0: the numerics of v_mfma_f32_16x16x4_f32 (k_tile_score)."""
    s = np.zeros(theta_rows.shape[0], dtype=F32)
    for k in range(theta_rows.shape[1]):
        s = fma_f32(theta_rows[:, k], phi_rows[:, k], s)
    return s


def score(theta, phi, d1, w1, d2=None, w2=None):
    s1 = dot_rows(theta[d1], phi[w1])
    if d2 is None:
        return s1, s1, None
    s2 = dot_rows(theta[d2], phi[w2])
    return np.minimum(s1, s2).astype(F32), s1, s2


# ------------------------------------------------------------------------------------------------
# slow textbook collapsed Gibbs (statistical cross-check only; not bitwise)
# ------------------------------------------------------------------------------------------------
def textbook_cgs(docs: list[np.ndarray], V: int, K: int, alpha: float, beta: float, sweeps: int, seed: int,
                 z0: list[np.ndarray] | None = None, on_sweep=None):
    """Slow, exact sequential collapsed Gibbs (Griffiths & Steyvers 2004): every count excludes
    the token being resampled, and every update is visible to the next token. ``z0`` is the
    initial assignment (default: uniform from ``seed``); ``on_sweep(sweep, z)`` is called after
    each sweep with the per-document topic arrays. Returns (z, n_dk, n_wk)."""
    rng = np.random.default_rng(seed)
    z = [np.array(a, dtype=np.int64) for a in z0] if z0 is not None else [rng.integers(0, K, size=len(d)) for d in docs]
    ndk = np.zeros((len(docs), K))
    nwk = np.zeros((V, K))
    for d, (ws, zs) in enumerate(zip(docs, z)):
        for w, t in zip(ws, zs):
            ndk[d, t] += 1
            nwk[w, t] += 1
    nk = nwk.sum(0)
    for sw in range(sweeps):
        for d, ws in enumerate(docs):
            for i, w in enumerate(ws):
                t = z[d][i]
                ndk[d, t] -= 1; nwk[w, t] -= 1; nk[t] -= 1
                p = (ndk[d] + alpha) * (nwk[w] + beta) / (nk + V * beta)
                c = np.cumsum(p)
                t = min(int(np.searchsorted(c, rng.random() * c[-1], side="right")), K - 1)
                z[d][i] = t
                ndk[d, t] += 1; nwk[w, t] += 1; nk[t] += 1
        if on_sweep is not None:
            on_sweep(sw + 1, z)
    return z, ndk, nwk
