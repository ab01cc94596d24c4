"""Proxy suspicious-connects (the `oni-ml YYYYMMDD proxy` path; SURVEY.md §2.2 C18, §2.8 "Proxy").

Bluecoat log → (C++ tokenizer) → columns → [GPU] host registered-domain/top-1M flag (K04),
user-agent frequency (K07: FNV hash → unique counts → per-event count), URI length + entropy (K06),
quantile cuts (K01) → word packing → corpus/LDA → score θ_client·φ_word → top-N.

Word (bit-packed u64, rendered ``top_tb_method_uab_ctype_eb_lb_respcode``):
  top(2b) @31 | time decile(4b) @27 | method code(4b) @23 | UA-frequency quintile(3b) @20 |
  content-type class(4b) @16 | URI-entropy quintile(3b) @13 | URI-length quintile(3b) @10 |
  response code(10b) @0
"""
from __future__ import annotations


import numpy as np
import torch

from .. import ops
from ..io import staging
from ..utils.obs import StageTimer, traced
from ..ops import strings as sops
from ..parallel.comm import Comm
from ..ref import spec
from ..store.columnar import StringColumn
from . import common
from .dns import top_set

METHODS = ["OTHER", "GET", "POST", "PUT", "HEAD", "CONNECT", "OPTIONS", "DELETE", "TRACE", "PATCH"]
CTYPE_CLASSES = [("", 0), ("-", 0), ("text/html", 1), ("text/", 2), ("image/", 3), ("application/javascript", 4),
                 ("application/json", 4), ("application/octet-stream", 5), ("application/", 6), ("video/", 7),
                 ("audio/", 8), ("multipart/", 9)]
BINNED = [("time", spec.DECILES, 27), ("ua_freq", spec.QUINTILES, 20), ("uri_ent", spec.QUINTILES, 13),
          ("uri_len", spec.QUINTILES, 10)]
RAW = [("method", 0xF, 23), ("ctype", 0xF, 16), ("respcode", 0x3FF, 0)]
TOP_SHIFT = 31


def ctype_class(s: str) -> int:
    s = s.strip().lower()
    best, blen = 10, -1
    for prefix, code in CTYPE_CLASSES:
        if (s == prefix if prefix in ("", "-") else s.startswith(prefix)) and len(prefix) > blen:
            best, blen = code, len(prefix)
    return best


def word_str(w: int) -> str:
    w = int(w)
    vals = {"top": (w >> TOP_SHIFT) & 3}
    for name, fr, s in BINNED:
        vals[name] = (w >> s) & (15 if fr is spec.DECILES else 7)
    for name, m, s in RAW:
        vals[name] = (w >> s) & m
    return "_".join(str(vals[k]) for k in ("top", "time", "method", "ua_freq", "ctype", "uri_ent", "uri_len", "respcode"))


STRING_COLS = ("host", "p_time", "useragent", "fulluri", "reqmethod", "resconttype")


def host_arrays(cols: dict) -> dict:
    """The host arrays the proxy model reads, in their device dtypes: ``<col>.off`` / ``<col>.chars``
    of the string columns, ``respcode``, ``clientip`` (a loader can pin and prefetch them,
    ``run_proxy(device_cols=...)``)."""
    out = {}
    for name in STRING_COLS:
        c: StringColumn = cols[name]
        out[name + ".off"] = c.offsets
        out[name + ".chars"] = c.chars if c.chars.size else np.zeros(1, np.uint8)
    out["respcode"] = np.asarray(cols["respcode"]).astype(np.int32, copy=False)
    out["clientip"] = np.asarray(cols["clientip"], np.uint32).view(np.int32)
    return out


def _codes_by_hash(col: StringColumn, off: torch.Tensor, ch: torch.Tensor, fn) -> torch.Tensor:
    """Categorical code per row via the distinct values only (few distinct methods / types)."""
    dev = off.device
    h, _, _ = sops.string_features(off, ch)
    uniq, first_idx, inv = _unique_first(h)
    labels = [fn(col[int(i)]) for i in first_idx.tolist()]
    table = torch.tensor(labels, dtype=torch.int32, device=dev)
    return table[inv].contiguous() if len(labels) else torch.zeros(0, dtype=torch.int32, device=dev)


def _unique_first(h: torch.Tensor):
    """(sorted unique values, first row of each (CPU), inverse). Sort-based: an atomic-min
    scatter_reduce here serialised 2M rows onto a handful of distinct values (27 ms per call)."""
    sh, order = torch.sort(h, stable=True)
    head = torch.ones_like(sh, dtype=torch.bool)
    if sh.numel() > 1:
        head[1:] = sh[1:] != sh[:-1]
    # group id of every sorted row by a scan over the run heads (repeat_interleave of the few run
    # lengths put one thread on each run: 436 µs per call on 2M rows with 5 distinct methods)
    grp = torch.cumsum(head, 0) - 1
    uniq, first = sh[head], order[head]
    inv = torch.empty_like(order)
    inv[order] = grp
    return uniq, first.cpu(), inv


# the same rules as method_code / ctype_class as device pattern tables (ops.strings.category_codes)
METHOD_PATTERNS = tuple((m, 0, i) for i, m in enumerate(METHODS))
CTYPE_PATTERNS = tuple((p, 0 if p in ("", "-") else 1, c) for p, c in CTYPE_CLASSES)


def method_code(s: str) -> int:
    s = s.strip().upper()
    return METHODS.index(s) if s in METHODS else 0


_HOUR_TABLES: dict = {}


def _hour_table(dev) -> torch.Tensor:
    """f32 (h + m/60) + s/3600 for every second of the day, computed on the host exactly as the
    word spec does, then kept on the device (a p_time → hour lookup)."""
    key = str(dev)
    if key not in _HOUR_TABLES:
        sod = np.arange(86400, dtype=np.int64)
        hh, mm, ss = sod // 3600, sod // 60 % 60, sod % 60
        t = (torch.from_numpy(hh.astype(np.float32)) + torch.from_numpy(mm.astype(np.float32)) / 60.0) \
            + torch.from_numpy(ss.astype(np.float32)) / 3600.0
        _HOUR_TABLES[key] = t.to(dev)
    return _HOUR_TABLES[key]


@traced("oni:proxy.featurize")
def featurize(cols: dict, device, comm: Comm | None, topset, allreduce_counts: bool = True, d: dict | None = None,
              day: tuple | None = None):
    """(words, cuts, UA table). ``d``: :func:`host_arrays` already on the device (else uploaded
    here). ``day`` = (cuts, UA table) of the day being scored: analyst feedback rows are worded
    with the day's cuts and the day's user-agent frequencies (a UA absent from the day counts 0),
    as the reference re-words feedback with the current model."""
    dev = torch.device(device)
    n = len(cols["clientip"])
    if d is None:
        d = {k: staging.upload(a, dev) for k, a in host_arrays(cols).items()}

    def strcol(name):
        return d[name + ".off"], d[name + ".chars"]

    ho, hc = strcol("host")
    _, top, _, _, _ = sops.domain_features(ho, hc, topset, "")
    # time of day from p_time "HH:MM:SS": the digits are read on the device, the f32 hour value
    # comes from a 86400-entry table built with the reference formula (bitwise the host result)
    po, pc = strcol("p_time")
    if n:
        base = po[:-1]
        ok = (po[1:] - base) >= 8  # malformed / short times read as 00:00:00
        last = pc.numel() - 1

        def dig(k):
            return torch.where(ok, pc[(base + k).clamp(max=last)].to(torch.int64) - 48, 0)
        sod = (dig(0) * 10 + dig(1)) * 3600 + (dig(3) * 10 + dig(4)) * 60 + (dig(6) * 10 + dig(7))
        t = _hour_table(dev)[sod.clamp_(0, 86399)]
    else:
        t = torch.zeros(0, dtype=torch.float32, device=dev)
    tkey = ops.f32_keys(t.contiguous())
    # K07: user-agent frequency over the day (global across ranks)
    uo, uc = strcol("useragent")
    uh, _, _ = sops.string_features(uo, uc)
    if day is not None:
        tk, tc = day[1]
        pos = torch.searchsorted(tk, uh).clamp_(max=max(tk.numel() - 1, 0))
        hit = tk[pos] == uh if tk.numel() else torch.zeros_like(uh, dtype=torch.bool)
        ua_freq = torch.where(hit, tc[pos] if tk.numel() else torch.zeros_like(uh), 0).clamp(max=2**31 - 1)
        ua_freq = ua_freq.to(torch.int32).contiguous()
        table = day[1]
    else:
        uq, inv, cnt = ua_histogram(uh)
        if comm is not None and comm.dist:
            keys = torch.cat(comm.allgather_var(uq))
            cnts = torch.cat(comm.allgather_var(cnt))
            gk, ginv = torch.unique(keys, return_inverse=True)
            gc = torch.zeros(gk.numel(), dtype=torch.int64, device=gk.device).index_add_(0, ginv, cnts.to(torch.int64))
            cnt = gc[torch.searchsorted(gk, uq.to(gk.device))].to(dev)
        ua_freq = cnt[inv.long()].clamp(max=2**31 - 1).to(torch.int32).contiguous()
        table = None
    fo, fc = strcol("fulluri")
    _, ulen, uent = sops.string_features(fo, fc)
    keys = {"time": tkey, "ua_freq": ua_freq, "uri_ent": ops.f32_keys(uent), "uri_len": ulen}
    if day is not None:
        cuts, dev_cuts = day[0], None
    else:
        n_glob = n
        if comm is not None and comm.dist:
            n_glob = int(comm.allreduce_np(np.array([n], np.int64))[0])
        cuts, dev_cuts = common.binned_cuts(keys, BINNED, comm, n_glob)
    if dev.type == "cuda":
        # per-row pattern match on the device: no distinct-value round trip through the host
        meth = sops.category_codes(*strcol("reqmethod"), METHOD_PATTERNS, 1, 0)
        ctyp = sops.category_codes(*strcol("resconttype"), CTYPE_PATTERNS, 2, 10)
    else:
        meth = _codes_by_hash(cols["reqmethod"], *strcol("reqmethod"), method_code)
        ctyp = _codes_by_hash(cols["resconttype"], *strcol("resconttype"), ctype_class)
    raws = {"method": meth, "ctype": ctyp,
            "respcode": d["respcode"]}
    words = sops.pack_words([keys[nm] for nm, _, _ in BINNED],
                            [range(len(fr)) if dev_cuts is not None else cuts[nm] for nm, fr, _ in BINNED],
                            [s for _, _, s in BINNED], [raws[nm] for nm, _, _ in RAW], [m for _, m, _ in RAW],
                            [s for _, _, s in RAW], raw8=top, r8mask=3, r8shift=TOP_SHIFT, dev_cuts=dev_cuts)
    if table is None:
        # the day's UA frequency table (signed-sorted keys, counts), for wording feedback rows
        ks, o = torch.sort(uq.to(dev) if comm is None or not comm.dist else uq)
        table = (ks, cnt[o].to(torch.int64))
    return words, cuts, table


def ua_histogram(uh: torch.Tensor):
    """K07: (distinct user-agent hashes, id of every row, count of every distinct hash). On the
    GPU one native radix pass (ops.corpus.dict_encode with run counts), no torch unique/bincount."""
    if uh.is_cuda:
        from ..ops import corpus as oc
        uq, inv, cnt = oc.dict_encode(uh.contiguous(), 64, counts=True)
        return uq, inv, cnt
    uq, inv, cnt = torch.unique(uh, return_inverse=True, return_counts=True)
    return uq, inv.to(torch.int32), cnt.to(torch.int64)


@traced("oni:proxy.run")
def run_proxy(cols: dict, K: int = 20, sweeps: int = 200, tol: float = 1.0, maxresults: int = 3000,
              alpha: float | None = None, beta: float | None = None, seed: int = 0x0D15EA5E, chunk_len: int = 0,
              device="cpu", comm: Comm | None = None, top_domains=None, feedback: dict | None = None,
              dupfactor: int = 1000, row_offset: int = 0, eval_every: int = 0, burnin: int = 0, ckpt=None,
              log=None, ldac_dir: str | None = None, ldac_lag: int = 0,
              device_cols: dict | None = None) -> common.SingleResult:
    """``device_cols``: :func:`host_arrays` already on the device (e.g. prefetched by
    io.staging.Prefetcher while the previous day computed)."""
    timer = StageTimer(device)
    with timer.stage("h2d"):
        d = dict(device_cols) if device_cols is not None else \
            {k: staging.upload(a, device) for k, a in host_arrays(cols).items()}
    with timer.stage("featurize"):
        topset = top_set(top_domains)
        words, cuts, ua_table = featurize(cols, device, comm, topset, d=d)
        docs = common.u32_to_i64(d["clientip"])
    fb = None
    if feedback and len(feedback.get("clientip", [])):
        fw, _, _ = featurize(feedback, device, None, topset, day=(cuts, ua_table))
        fdoc = torch.from_numpy(np.asarray(feedback["clientip"], np.uint32).astype(np.int64)).to(words.device)
        fb = (fdoc, fw, torch.full_like(fw, int(dupfactor)))
    res = common.run_single_doc_events(docs, words, K, sweeps, tol, maxresults, alpha, beta, seed, chunk_len, comm,
                                       feedback=fb, row_offset=row_offset, eval_every=eval_every, burnin=burnin, ckpt=ckpt, log=log,
                                       timer=timer, ldac_dir=ldac_dir, ldac_lag=ldac_lag,
                                       key_bits=34)
    res.stats["cuts"] = {k: [int(x) for x in v] for k, v in cuts.items()}
    return res
