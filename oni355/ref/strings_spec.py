"""NumPy/Python oracle for the string kernels (csrc/kernels/strings.hip, pack_words.hip).

Bit-exact mirror: FNV-1a over lowercased bytes, the 64-bin character classes, the f32 entropy
tables and their summation order, the public-suffix rule (psl.py), the open-addressing set.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32
FNV_OFF = 1469598103934665603
FNV_PRIME = 1099511628211
M64 = (1 << 64) - 1


def tables() -> tuple[np.ndarray, np.ndarray]:
    """clogc[c] = c·log2(c), lg[n] = log2(n) as f32 (c, n in 0..255); index 0 -> 0."""
    clogc = np.array([0.0] + [c * math.log2(c) for c in range(1, 256)], dtype=np.float64).astype(F32)
    lg = np.array([0.0] + [math.log2(n) for n in range(1, 256)], dtype=np.float64).astype(F32)
    return clogc, lg


_CLOGC, _LG = tables()


def _lower(b: bytes) -> bytes:
    return bytes(c + 32 if 65 <= c <= 90 else c for c in b)


def fnv1a(b: bytes) -> int:
    h = FNV_OFF
    for c in _lower(b):
        h = ((h ^ c) * FNV_PRIME) & M64
    return h


def cbin(c: int) -> int:
    if 97 <= c <= 122:
        return c - 97
    if 48 <= c <= 57:
        return 26 + c - 48
    if c == 45:
        return 36
    if c == 95:
        return 37
    if c == 46:
        return 38
    return 39 + c % 25


def entropy(b: bytes) -> np.float32:
    n = len(b)
    if n <= 0:
        return F32(0.0)
    h = [0] * 64
    for c in _lower(b):
        h[cbin(c)] = (h[cbin(c)] + 1) & 0xFF
    s = F32(0.0)
    for k in range(64):
        s = F32(s + _CLOGC[h[k]])
    return F32(_LG[min(n, 255)] - F32(s / F32(n)))


def split_domain(name: bytes, rules=None) -> tuple[int, int, int]:
    """(registered-domain start, end, periods) for a name (trailing dots stripped); the
    registered domain is the public suffix (oni355/ref/psl.py rules) plus one label."""
    from .psl import registered_start
    b = len(name)
    while b > 0 and name[b - 1] == 46:
        b -= 1
    per = sum(1 for j in range(b) if name[j] == 46)
    return registered_start(name, b, rules), b, per


class HashSet:
    """Open-addressing set of u64 hashes (0 = empty), power-of-two table, linear probe."""

    def __init__(self, hashes, load: float = 0.5):
        hs = np.unique(np.asarray(hashes, dtype=np.uint64))
        cap = 1
        while cap < max(2, int(len(hs) / load)):
            cap <<= 1
        self.mask = cap - 1
        tab = np.zeros(cap, dtype=np.uint64)
        for h in hs.tolist():
            h = h or 1
            i = (h ^ (h >> 29)) & self.mask
            while tab[i] != 0 and int(tab[i]) != h:
                i = (i + 1) & self.mask
            tab[i] = h
        self.table = tab

    def __contains__(self, h: int) -> bool:
        h = int(h) or 1
        i = (h ^ (h >> 29)) & self.mask
        for _ in range(min(self.mask + 1, 4096)):
            v = int(self.table[i])
            if v == h:
                return True
            if v == 0:
                return False
            i = (i + 1) & self.mask
        return False


def domain_features(offsets, chars, topset: HashSet | None, user_domain: str = "", rules=None):
    offsets = np.asarray(offsets, dtype=np.int64)
    raw = bytes(np.asarray(chars, dtype=np.uint8))
    n = offsets.size - 1
    uh = fnv1a(user_domain.encode()) if user_domain else 0
    user_is_label = "." not in user_domain
    reg_hash = np.zeros(n, np.uint64)
    top = np.zeros(n, np.uint8)
    sub_len = np.zeros(n, np.int32)
    ent = np.zeros(n, np.float32)
    per = np.zeros(n, np.int32)
    for i in range(n):
        name = raw[offsets[i]:offsets[i + 1]]
        reg, b, p = split_domain(name, rules)
        sub_end = reg - 1 if reg > 0 else 0
        rh = fnv1a(name[reg:b])
        lab_end = reg
        while lab_end < b and name[lab_end] != 46:
            lab_end += 1
        lh = fnv1a(name[reg:lab_end])
        t = 0
        if uh and (lh == uh if user_is_label else rh == uh):
            t = 2
        elif topset is not None and rh in topset:
            t = 1
        reg_hash[i], top[i], sub_len[i], per[i] = rh, t, sub_end, p
        ent[i] = entropy(name[:sub_end])
    return reg_hash, top, sub_len, ent, per


def string_features(offsets, chars):
    offsets = np.asarray(offsets, dtype=np.int64)
    raw = bytes(np.asarray(chars, dtype=np.uint8))
    n = offsets.size - 1
    h = np.zeros(n, np.uint64)
    ln = np.zeros(n, np.int32)
    en = np.zeros(n, np.float32)
    for i in range(n):
        s = raw[offsets[i]:offsets[i + 1]]
        h[i] = fnv1a(s)
        ln[i] = len(s)
        en[i] = entropy(s[:255])
    return h, ln, en


def pack_words(keys, cuts, kshift, raws, rmask, rshift, raw8=None, r8mask=0, r8shift=0) -> np.ndarray:
    n = len(keys[0]) if keys else len(raws[0])
    w = np.zeros(n, dtype=np.uint64)
    for k, c, s in zip(keys, cuts, kshift):
        b = (np.asarray(k, np.uint32)[:, None] > np.asarray(c, np.uint32)[None, :]).sum(1).astype(np.uint64)
        w |= b << np.uint64(s)
    for r, m, s in zip(raws, rmask, rshift):
        w |= (np.asarray(r).astype(np.int64).astype(np.uint32) & np.uint32(m)).astype(np.uint64) << np.uint64(s)
    if raw8 is not None:
        w |= (np.asarray(raw8, np.uint8) & np.uint8(r8mask)).astype(np.uint64) << np.uint64(r8shift)
    return w
