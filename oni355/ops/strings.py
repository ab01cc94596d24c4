"""String/word-packing device ops (DNS & proxy featurization), CPU → oracle, CUDA → HIP kernels."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ..ref import strings_spec as ss
from . import _lib

vp, i64 = C.c_void_p, C.c_int64
K_MAX_BINNED, K_MAX_RAW, K_MAX_CUTS = 8, 4, 15


class OniPack(C.Structure):
    _fields_ = [
        ("key", vp * K_MAX_BINNED), ("ncuts", C.c_int32 * K_MAX_BINNED), ("kshift", C.c_int32 * K_MAX_BINNED),
        ("cuts", (C.c_uint32 * K_MAX_CUTS) * K_MAX_BINNED), ("raw", vp * K_MAX_RAW),
        ("rmask", C.c_uint32 * K_MAX_RAW), ("rshift", C.c_int32 * K_MAX_RAW), ("raw8", vp), ("r8mask", C.c_uint32),
        ("r8shift", C.c_int32), ("nkeys", C.c_int32), ("nraw", C.c_int32), ("n", C.c_int64), ("out", vp),
        ("dcuts", vp),
    ]


_lib.register_optional("oni_domain_features", [vp, vp, i64, vp, C.c_uint64, C.c_uint64, C.c_int, vp, vp,
                                               vp, C.c_uint64, vp, C.c_uint64, C.c_int,
                                               vp, vp, vp, vp, vp, vp])
_lib.register_optional("oni_string_features", [vp, vp, i64, vp, vp, vp, vp, vp, vp])
_lib.register_optional("oni_set_probe", [vp, i64, vp, C.c_uint64, vp, vp])
_lib.register_optional("oni_pack_words", [C.POINTER(OniPack), vp])
_lib.register_optional("oni_category_codes", [vp, vp, i64, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, vp])
_lib.register_optional("oni_pack_sizeof", [])

_tables: dict = {}


def _dev_psl(device, rules):
    """The rule and exception hash tables of ``rules`` on ``device``, cached on the rules object
    itself (an id()-keyed module cache could hand a new object the tables of a collected one)."""
    cache = rules.__dict__.setdefault("_dev_tables", {})
    key = str(device)
    if key not in cache:
        cache[key] = (torch.from_numpy(rules.rule_set.table.view(np.int64)).to(device),
                      torch.from_numpy(rules.exc_set.table.view(np.int64)).to(device))
    return cache[key]


def _dev_tables(device):
    key = str(device)
    if key not in _tables:
        clogc, lg = ss.tables()
        _tables[key] = (torch.from_numpy(clogc).to(device), torch.from_numpy(lg).to(device))
    return _tables[key]


def _u64(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


def _dev_topset(topset, dev) -> torch.Tensor:
    """The hash set's table on ``dev``, uploaded once per set object and device."""
    cache = topset.__dict__.setdefault("_dev_tables", {})
    key = str(dev)
    if key not in cache:
        cache[key] = torch.from_numpy(topset.table.view(np.int64)).to(dev)
    return cache[key]


def domain_features(offsets: torch.Tensor, chars: torch.Tensor, topset: ss.HashSet | None, user_domain: str = "",
                    rules=None):
    """Returns (reg_hash int64(u64 bits), top u8, sub_len i32, sub_ent f32, periods i32).
    ``rules``: public-suffix rules (oni355.ref.psl.SuffixRules; default: the built-in list)."""
    from ..ref import psl
    rules = rules or psl.default_rules()
    n = offsets.numel() - 1
    if offsets.device.type != "cuda":
        rh, top, sl, en, per = ss.domain_features(offsets.numpy(), chars.numpy(), topset, user_domain, rules)
        return (torch.from_numpy(rh.view(np.int64)), torch.from_numpy(top), torch.from_numpy(sl),
                torch.from_numpy(en), torch.from_numpy(per))
    dev = offsets.device
    clogc, lg = _dev_tables(dev)
    tab = _dev_topset(topset, dev) if topset is not None else None
    mask = topset.mask if topset is not None else 0
    uh = ss.fnv1a(user_domain.encode()) if user_domain else 0
    outs = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.uint8, device=dev),
            torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.float32, device=dev),
            torch.empty(n, dtype=torch.int32, device=dev))
    ch = chars if chars.numel() else torch.zeros(1, dtype=torch.uint8, device=dev)
    prt, pet = _dev_psl(dev, rules)
    _lib.check(_lib.lib().oni_domain_features(_lib.ptr(offsets), _lib.ptr(ch), n, _lib.ptr(tab), mask, uh,
                                              1 if "." not in user_domain else 0, _lib.ptr(clogc), _lib.ptr(lg),
                                              _lib.ptr(prt), rules.rule_set.mask, _lib.ptr(pet), rules.exc_set.mask,
                                              rules.max_labels, *map(_lib.ptr, outs), _lib.stream()),
               "oni_domain_features")
    return outs


def string_features(offsets: torch.Tensor, chars: torch.Tensor):
    """(hash int64(u64 bits), length i32, entropy f32) per string."""
    n = offsets.numel() - 1
    if offsets.device.type != "cuda":
        h, ln, en = ss.string_features(offsets.numpy(), chars.numpy())
        return torch.from_numpy(h.view(np.int64)), torch.from_numpy(ln), torch.from_numpy(en)
    dev = offsets.device
    clogc, lg = _dev_tables(dev)
    outs = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
            torch.empty(n, dtype=torch.float32, device=dev))
    ch = chars if chars.numel() else torch.zeros(1, dtype=torch.uint8, device=dev)
    _lib.check(_lib.lib().oni_string_features(_lib.ptr(offsets), _lib.ptr(ch), n, _lib.ptr(clogc), _lib.ptr(lg),
                                              *map(_lib.ptr, outs), _lib.stream()), "oni_string_features")
    return outs


def _split_cuts(flat: np.ndarray, sizes: list) -> list:
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    return [flat[off[i]:off[i + 1]] for i in range(len(sizes))]


def pack_words(keys: list, cuts: list, kshift: list, raws: list, rmask: list, rshift: list, raw8=None, r8mask=0,
               r8shift=0, dev_cuts: torch.Tensor | None = None) -> torch.Tensor:
    """Word keys (int64 holding u64 bits) from binned order keys + raw categorical fields.
    ``dev_cuts``: the cut lists already on the device, concatenated (int32 bits); ``cuts`` then
    only gives each list's length."""
    ref = keys[0] if keys else raws[0]
    n = ref.numel()
    if dev_cuts is not None and ref.device.type != "cuda":
        dev_cuts, cuts = None, _split_cuts(dev_cuts.numpy().view(np.uint32), [len(c) for c in cuts])
    if ref.device.type != "cuda":
        w = ss.pack_words([k.numpy().view(np.uint32) for k in keys], cuts, kshift, [r.numpy() for r in raws], rmask,
                          rshift, None if raw8 is None else raw8.numpy(), r8mask, r8shift)
        return torch.from_numpy(w.view(np.int64))
    a = OniPack()
    if dev_cuts is not None:
        if dev_cuts.dtype != torch.int32 or dev_cuts.numel() != sum(len(c) for c in cuts):
            raise ValueError("dev_cuts: int32 concatenation of every binned component's cut list")
        a.dcuts = _lib.ptr(dev_cuts)
    for i, (k, c, s) in enumerate(zip(keys, cuts, kshift)):
        if dev_cuts is None:
            c = np.asarray(c, np.uint32)
        if len(c) > K_MAX_CUTS or k.dtype != torch.int32 or k.numel() != n:
            raise ValueError("bad binned component")
        a.key[i] = _lib.ptr(k)
        a.ncuts[i] = len(c)
        a.kshift[i] = s
        if dev_cuts is None:
            for j, v in enumerate(c.tolist()):
                a.cuts[i][j] = v
    for i, (r, m, s) in enumerate(zip(raws, rmask, rshift)):
        if r.dtype != torch.int32 or r.numel() != n:
            raise ValueError("raw components must be int32 of length n")
        a.raw[i] = _lib.ptr(r)
        a.rmask[i] = m
        a.rshift[i] = s
    if raw8 is not None:
        a.raw8, a.r8mask, a.r8shift = _lib.ptr(raw8), r8mask, r8shift
    a.nkeys, a.nraw, a.n = len(keys), len(raws), n
    out = torch.empty(n, dtype=torch.int64, device=ref.device)
    a.out = _lib.ptr(out)
    L = _lib.lib()
    if L.oni_pack_sizeof() != C.sizeof(OniPack):
        raise RuntimeError("OniPack ABI mismatch; rebuild")
    _lib.check(L.oni_pack_words(C.byref(a), _lib.stream()), "oni_pack_words")
    return out


def _category_table(patterns: tuple, device):
    """Device pattern table of :func:`category_codes` (cached per pattern tuple and device)."""
    key = (patterns, str(device))
    if key not in _tables:
        if len(patterns) > 32 or any(len(p.encode()) > 32 for p, _, _ in patterns):
            raise ValueError("category patterns: at most 32, of at most 32 bytes")
        pat = np.zeros((max(len(patterns), 1), 32), np.uint8)
        for i, (p, _, _) in enumerate(patterns):
            b = p.encode()
            pat[i, :len(b)] = np.frombuffer(b, np.uint8)
        cols = [np.array([len(p.encode()) for p, _, _ in patterns] or [0], np.int32),
                np.array([m for _, m, _ in patterns] or [0], np.int32),
                np.array([c for _, _, c in patterns] or [0], np.int32)]
        _tables[key] = (torch.from_numpy(pat.reshape(-1)).to(device), *(torch.from_numpy(c).to(device) for c in cols))
    return _tables[key]


def category_codes(offsets: torch.Tensor, chars: torch.Tensor, patterns: tuple, fold: int, default: int) -> torch.Tensor:
    """int32 code per string (k_category_codes): trim ASCII whitespace, fold case (1 upper, 2 lower),
    then the code of the longest matching pattern ((text, mode 0 exact / 1 prefix, code), first
    of equal length wins), else ``default``. GPU only (the CPU path labels distinct values)."""
    n = offsets.numel() - 1
    dev = offsets.device
    out = torch.empty(max(n, 0), dtype=torch.int32, device=dev)
    if n <= 0:
        return out
    pat, plen, pmode, pcode = _category_table(tuple(patterns), dev)
    ch = chars if chars.numel() else torch.zeros(1, dtype=torch.uint8, device=dev)
    _lib.check(_lib.lib().oni_category_codes(_lib.ptr(offsets), _lib.ptr(ch), n, _lib.ptr(pat), _lib.ptr(plen),
                                             _lib.ptr(pmode), _lib.ptr(pcode), len(patterns), int(fold), int(default),
                                             _lib.ptr(out), _lib.stream()), "oni_category_codes")
    return out
