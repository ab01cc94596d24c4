"""DNS suspicious-connects (the `oni-ml YYYYMMDD dns` path; SURVEY.md §3.4, §2.8 "DNS").

pcap → (C++ decoder) → columns → [GPU] domain features (K04: registered domain with ccTLD rule,
user-domain / top-1M flag, subdomain length + entropy, dot count) → quantile cuts (K01) →
word packing (K05) → corpus/LDA (K=50 by default) → score θ_client·φ_word → top-N.

Word (table-driven, bit-packed u64; rendered ``top_flb_tb_slb_eb_pb_qtype_rcode``):
  top(2b) @37 | frame_len decile(4b) @33 | time decile(4b) @29 | subdomain-length quintile(3b) @26 |
  subdomain-entropy quintile(3b) @23 | periods quintile(3b) @20 | qtype(16b) @4 | rcode(4b) @0
Document = ``ip_dst`` (the client receiving the response).
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
from ..ref.strings_spec import HashSet, fnv1a
from ..store.columnar import StringColumn
from . import common

# (component, fractions, shift) -- the DNS word layout
BINNED = [("frame_len", spec.DECILES, 33), ("time", spec.DECILES, 29), ("sub_len", spec.QUINTILES, 26),
          ("sub_ent", spec.QUINTILES, 23), ("periods", spec.QUINTILES, 20)]
RAW = [("dns_qry_type", 0xFFFF, 4), ("dns_qry_rcode", 0xF, 0)]
TOP_SHIFT = 37


def word_str(w: int) -> str:
    w = int(w)
    parts = [(w >> TOP_SHIFT) & 3] + [(w >> s) & (15 if fr is spec.DECILES else 7) for _, fr, s in BINNED]
    parts += [(w >> s) & m for _, m, s in RAW]
    return "_".join(str(p) for p in parts)


_TOP_CACHE: list = []  # [(domains object, HashSet)]: one entry, the list the pipeline keeps passing


def top_set(domains) -> HashSet | None:
    """Top-domain hash set of ``domains`` (built once per list object: hashing and inserting a
    top-1M list in Python takes seconds, and every day of a run passes the same list)."""
    if not domains:
        return None
    if _TOP_CACHE and _TOP_CACHE[0][0] is domains and _TOP_CACHE[0][2] == len(domains):
        return _TOP_CACHE[0][1]
    hs = HashSet([fnv1a(d.strip().lower().encode()) for d in domains if d.strip()])
    _TOP_CACHE[:] = [(domains, hs, len(domains))]
    return hs


def load_top_domains(path: str) -> list[str]:
    """Alexa-style ``rank,domain`` CSV (or one domain per line)."""
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line:
                out.append(line.split(",")[-1])
    return out


def host_arrays(cols: dict) -> dict:
    """The host arrays the DNS model reads, in their device dtypes (what :func:`to_device` uploads;
    a loader can pin and prefetch them, ``run_dns(device_cols=...)``)."""
    d = {"unix_tstamp": np.asarray(cols["unix_tstamp"], np.int64)}
    for k in ("frame_len", "dns_qry_type", "dns_qry_rcode"):
        d[k] = np.asarray(cols[k]).astype(np.int32, copy=False)
    d["ip_dst"] = np.asarray(cols["ip_dst"], np.uint32).view(np.int32)
    nm: StringColumn = cols["dns_qry_name"]
    d["name_off"] = nm.offsets
    d["name_chars"] = nm.chars if nm.chars.size else np.zeros(1, np.uint8)
    return d


def to_device(cols: dict, device) -> dict:
    return {k: staging.upload(a, device) for k, a in host_arrays(cols).items()}


def time_keys(unix: torch.Tensor) -> torch.Tensor:
    """f32 order key of hour + min/60 + sec/3600 (UTC), same arithmetic as the flow kernel."""
    sec = torch.remainder(unix, 86400)
    h = (sec // 3600).to(torch.float32)
    m = (sec // 60 % 60).to(torch.float32)
    s = (sec % 60).to(torch.float32)
    t = (h + m / 60.0) + s / 3600.0
    return ops.f32_keys(t.contiguous())


@traced("oni:dns.featurize")
def featurize(d: dict, comm: Comm | None, topset: HashSet | None, user_domain: str):
    rh, top, sub_len, sub_ent, per = sops.domain_features(d["name_off"], d["name_chars"], topset, user_domain)
    keys = {"frame_len": d["frame_len"], "time": time_keys(d["unix_tstamp"]), "sub_len": sub_len,
            "sub_ent": ops.f32_keys(sub_ent), "periods": per}
    n = d["frame_len"].numel()
    n_glob = n
    if comm is not None and comm.dist:
        n_glob = int(comm.allreduce_np(np.array([n], np.int64))[0])
    cuts, dev_cuts = common.binned_cuts(keys, BINNED, comm, n_glob)
    words = sops.pack_words([keys[name].contiguous() for name, _, _ in BINNED],
                            [range(len(fr)) if dev_cuts is not None else cuts[name] for name, fr, _ in BINNED],
                            [s for _, _, s in BINNED], [d[name] for name, _, _ in RAW], [m for _, m, _ in RAW],
                            [s for _, _, s in RAW], raw8=top, r8mask=3, r8shift=TOP_SHIFT, dev_cuts=dev_cuts)
    feats = {"top": top, "sub_len": sub_len, "sub_ent": sub_ent, "periods": per, "reg_hash": rh}
    return words, cuts, feats


@traced("oni:dns.run")
def run_dns(cols: dict, K: int = 50, sweeps: int = 200, tol: float = 1.0, maxresults: int = 3000,
            alpha: float | None = None, beta: float | None = None, seed: int = 0x0D15EA5E, chunk_len: int = 0,
            device="cpu", comm: Comm | None = None, top_domains=None, user_domain: str = "",
            feedback: dict | None = None, dupfactor: int = 1000, row_offset: int = 0, eval_every: int = 0, burnin: int = 0,
            ckpt=None, log=None, ldac_dir: str | None = None, ldac_lag: int = 0,
            device_cols: dict | None = None) -> common.SingleResult:
    """``device_cols``: :func:`host_arrays` already on the device (e.g. prefetched by
    io.staging.Prefetcher while the previous day computed)."""
    timer = StageTimer(device)
    with timer.stage("h2d"):
        d = dict(device_cols) if device_cols is not None else to_device(cols, device)
    with timer.stage("featurize"):
        topset = top_set(top_domains)
        words, cuts, feats = featurize(d, comm, topset, user_domain)
    docs = common.u32_to_i64(d["ip_dst"])
    fb = None
    if feedback and len(feedback.get("ip_dst", [])):
        fd = to_device(feedback, device)
        # feedback rows are re-worded with the CURRENT day's cuts (reference behaviour, C19)
        rh, top, sl, se, per = sops.domain_features(fd["name_off"], fd["name_chars"], topset, user_domain)
        fk = {"frame_len": fd["frame_len"], "time": time_keys(fd["unix_tstamp"]), "sub_len": sl,
              "sub_ent": ops.f32_keys(se), "periods": per}
        fw = sops.pack_words([fk[name].contiguous() for name, _, _ in BINNED], [cuts[name] for name, _, _ in BINNED],
                             [s for _, _, s in BINNED], [fd[name] for name, _, _ in RAW], [m for _, m, _ in RAW],
                             [s for _, _, s in RAW], raw8=top, r8mask=3, r8shift=TOP_SHIFT)
        fdoc = common.u32_to_i64(fd["ip_dst"])
        fb = (fdoc, fw, torch.full_like(fw, int(dupfactor)))
    res = common.run_single_doc_events(docs, words, K, sweeps, tol, maxresults, alpha, beta, seed, chunk_len, comm,
                                       feedback=fb, row_offset=row_offset, eval_every=eval_every, burnin=burnin, ckpt=ckpt, log=log,
                                       timer=timer, ldac_dir=ldac_dir, ldac_lag=ldac_lag,
                                       key_bits=40)
    res.stats["cuts"] = {k: [int(x) for x in v] for k, v in cuts.items()}
    res.stats["features"] = feats
    return res
