"""Netflow suspicious-connects (the `oni-ml YYYYMMDD flow` path).

Stages (each a device op; see csrc/kernels):
  K01  quantile cuts: deciles(time), deciles(ibyt), quintiles(ipkt)   (radix select, X03 in DP)
  K03  flow word creation (port rule + bins, two word keys per flow)
  K08/K09 vocabulary, owner routing, CSR + SELL corpus (+ feedback dupes ×DUPFACTOR)
  K10-K12 collapsed-Gibbs sweeps (+ RCCL all-reduce of Δn_wk per sweep)
  K13/K15/K16 θ/φ, per-flow score = min(θ_sip·φ_srcw, θ_dip·φ_dstw), top-N below TOL

Reference call stack being replaced: ml_ops.sh → spark-submit SuspiciousConnects (FlowPreLDA,
OniLDACWrapper/mpiexec lda est, FlowPostLDA) → getmerge flow_results.csv ([U-M]).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..io import staging
from ..utils.obs import StageTimer, traced
from ..parallel.comm import Comm
from ..ref import spec
from . import common

DEVICE_COLS = {"trhour": torch.int32, "trminute": torch.int32, "trsec": torch.int32, "ibyt": torch.int64,
               "ipkt": torch.int64, "sport": torch.int32, "dport": torch.int32, "sip": torch.int32,
               "dip": torch.int32}


# IPv6 documents: every distinct IPv6 address of the day gets the 32-bit key V6_KEY_BASE + its
# rank in the day's sorted IPv6 dictionary (exact, identical on every rank). 240.0.0.0/4 is the
# reserved, never-routed IPv4 block, so the keys cannot collide with a real IPv4 document.
V6_KEY_BASE = 0xF0000000
V6_KEY_MAX = 1 << 28
V6_KEYED = "_v6_keyed"  # marker left in columns that went through with_ipv6_keys


def _needs_v6_keys(c: dict | None) -> bool:
    return bool(c) and any(k in c for k in ("sip6", "dip6")) and not c.get(V6_KEYED, False)


def _fixed(col, w: int = 48) -> np.ndarray:
    """StringColumn → fixed-width bytes array (dtype S<w>), vectorised."""
    off = col.offsets
    ln = np.minimum(np.diff(off), w)
    m = np.zeros((len(col), w), np.uint8)
    if ln.sum():
        r = np.repeat(np.arange(len(col)), ln)
        k = np.arange(int(ln.sum())) - np.repeat(np.cumsum(ln) - ln, ln)
        m[r, k] = col.chars[np.repeat(off[:-1], ln) + k]
    return m.view(f"S{w}").reshape(-1)


def ip4(x: int) -> str:
    return "%d.%d.%d.%d" % (x >> 24, (x >> 16) & 255, (x >> 8) & 255, x & 255)


def with_ipv6_keys(cols: dict, comm: Comm | None = None, others: tuple = ()) -> dict:
    """Columns with ``sip``/``dip`` of IPv6 rows replaced by their day-dictionary keys
    (:data:`V6_KEY_BASE` + rank); ``others`` (e.g. analyst feedback rows) share the dictionary and
    are returned keyed too. On such a day, IPv4 addresses inside 240.0.0.0/4 (bogons) go through
    the dictionary as well, so no IPv4 document can share a key with an IPv6 one; their dotted
    text lands in ``sip6``/``dip6`` for rendering. No IPv6 columns anywhere: the inputs come back
    unchanged."""
    sets = [c for c in (cols, *others) if c]
    have = any(k in c for c in sets for k in ("sip6", "dip6"))
    if comm is not None and comm.dist:
        have = comm.allreduce_scalar(1.0 if have else 0.0, "max") > 0
    if not have:
        return cols if not others else (cols, *others)

    def text(c: dict, k4: str, k6: str):
        """Fixed-width dictionary text of the rows keyed through the dictionary: IPv6 rows, and
        IPv4 rows inside 240.0.0.0/4 (class-E bogons would otherwise share the IPv6 key space)."""
        v4 = np.asarray(c[k4]).astype(np.uint32) if k4 in c else None
        f = _fixed(c[k6]) if k6 in c else (np.zeros(v4.size, "S48") if v4 is not None else None)
        if v4 is not None:
            ce = (f == b"") & (v4 >= np.uint32(V6_KEY_BASE))
            if ce.any():
                f = f.copy()
                f[ce] = np.array([("v4:%d.%d.%d.%d" % (x >> 24, (x >> 16) & 255, (x >> 8) & 255, x & 255)).encode()
                                  for x in v4[ce].tolist()], "S48")
        return f

    parts = []
    for c in sets:
        for k4, k6 in (("sip", "sip6"), ("dip", "dip6")):
            if k6 in c or k4 in c:
                f = text(c, k4, k6)
                parts.append(f[f != b""])
    uniq = np.unique(np.concatenate(parts)) if parts else np.zeros(0, "S48")
    if comm is not None and comm.dist:
        import torch.distributed as dist
        allp = [None] * comm.world
        dist.all_gather_object(allp, uniq.tolist(), group=comm.group)
        uniq = np.unique(np.array([x for p in allp for x in p], dtype="S48"))
    if uniq.size >= V6_KEY_MAX:
        raise ValueError(f"{uniq.size} distinct IPv6 addresses exceed the 2^28 key space")

    def keyed(c: dict) -> dict:
        from ..store.columnar import StringColumn
        out = dict(c)
        out[V6_KEYED] = True
        for k4, k6 in (("sip", "sip6"), ("dip", "dip6")):
            if k4 not in c:
                continue
            f = text(c, k4, k6)
            v6 = f != b""
            key = (V6_KEY_BASE + np.searchsorted(uniq, f)).astype(np.uint32)
            out[k4] = np.where(v6, key, np.asarray(c[k4]).astype(np.uint32))
            v4 = np.asarray(c[k4]).astype(np.uint32)
            no6 = (_fixed(c[k6]) == b"") if k6 in c else np.ones(v4.size, bool)
            ce = v6 & no6 & (v4 >= np.uint32(V6_KEY_BASE))
            if k6 not in c:
                if ce.any():  # class-E rows render their dotted address from the text column
                    out[k6] = StringColumn.from_list([ip4(x) if m else "" for x, m in zip(v4.tolist(), ce.tolist())])
            elif ce.any():
                t = c[k6].to_list()
                out[k6] = StringColumn.from_list([ip4(x) if m else s6 for s6, x, m in zip(t, v4.tolist(), ce.tolist())])
        return out

    res = [keyed(c) if c else c for c in (cols, *others)]
    return res[0] if not others else tuple(res)


def to_device(cols: dict, device) -> dict:
    """Host columns → device through the pinned staging ring (io/staging.py): the host-side
    dtype conversion of column j+1 overlaps the DMA of column j."""
    out = {}
    for name, dt in DEVICE_COLS.items():
        a = np.asarray(cols[name])
        if a.dtype == np.uint32:
            a = a.view(np.int32)
        out[name] = staging.upload(a, device, dt)
    return out


class FlowCuts:
    """The day's quantile cuts (time deciles, ibyt deciles, ipkt quintiles). On a GPU they are
    computed and consumed on the device (``dev``: the three arrays concatenated, int32 bits); the
    host arrays are fetched only if something reads them."""

    def __init__(self, time=None, ibyt=None, ipkt=None, dev: torch.Tensor | None = None, sizes=(9, 9, 4)):
        self._host = None if time is None else (np.asarray(time), np.asarray(ibyt), np.asarray(ipkt))
        self.dev = dev
        self.sizes = tuple(sizes) if self._host is None else tuple(len(x) for x in self._host)

    def _h(self):
        if self._host is None:
            a = self.dev.cpu().numpy().view(np.uint32)
            t, b = self.sizes[0], self.sizes[0] + self.sizes[1]
            self._host = (a[:t].copy(), a[t:b].copy(), a[b:].copy())
        return self._host

    time = property(lambda self: self._h()[0])
    ibyt = property(lambda self: self._h()[1])
    ipkt = property(lambda self: self._h()[2])

    def as_dict(self) -> dict:
        return {"time": [float(x) for x in spec.key_f32(self.time)], "ibyt": [int(x) for x in self.ibyt],
                "ipkt": [int(x) for x in self.ipkt]}


@traced("oni:flow.quantile_cuts")
def compute_cuts(d: dict, comm: Comm | None) -> FlowCuts:
    tk, bk, pk = ops.flow_keys(d["trhour"], d["trminute"], d["trsec"], d["ibyt"], d["ipkt"])
    n = tk.numel()
    ar = None
    n_glob = n
    if comm is not None and comm.dist:
        ar = comm.allreduce_np
        n_glob = int(comm.allreduce_np(np.array([n], dtype=np.int64))[0])
    fr = [spec.DECILES, spec.DECILES, spec.QUINTILES]
    if tk.is_cuda:
        # radix select entirely on the stream (X03: the histograms are all-reduced on the device)
        dev_ar = comm.allreduce_ if comm is not None and comm.dist else None
        cuts = FlowCuts(dev=ops.quantile_cuts_dev([tk, bk, pk], fr, dev_ar, n_glob), sizes=[len(f) for f in fr])
    else:
        cuts = FlowCuts(*ops.quantile_cuts_multi([tk, bk, pk], fr, ar, n_glob))
    d["_keys"] = (tk, bk, pk)
    return cuts


@traced("oni:flow.wordify")
def wordify(d: dict, cuts: FlowCuts) -> tuple[torch.Tensor, torch.Tensor]:
    tk, bk, pk = d.get("_keys") or ops.flow_keys(d["trhour"], d["trminute"], d["trsec"], d["ibyt"], d["ipkt"])
    if cuts.dev is not None and tk.is_cuda:
        nt, nb, npk = cuts.sizes
        return ops.flow_wordify(d["sport"], d["dport"], tk, bk, pk, range(nt), range(nb), range(npk),
                                dev_cuts=cuts.dev)
    return ops.flow_wordify(d["sport"], d["dport"], tk, bk, pk, cuts.time, cuts.ibyt, cuts.ipkt)


@dataclass
class FlowResult:
    rows: np.ndarray           # global row ids, ascending score
    scores: np.ndarray
    src_scores: np.ndarray
    dst_scores: np.ndarray
    src_words: np.ndarray      # packed word keys of the result rows
    dst_words: np.ndarray
    cuts: FlowCuts
    timings: dict = field(default_factory=dict)
    stats: dict = field(default_factory=dict)
    lda: object = None


def feedback_tokens(fb_cols: dict | None, cuts: FlowCuts, device, dupfactor: int):
    """sev==3 analyst rows → (doc keys, word keys, weights): each word duplicated DUPFACTOR times
    on its IP document (the reference's "noise filter"), as a count bump."""
    if not fb_cols or len(fb_cols.get("sip", [])) == 0:
        return None
    d = to_device(fb_cols, device)
    sw, dw = wordify({k: v for k, v in d.items()}, cuts)
    docs = torch.cat([common.u32_to_i64(d["sip"]), common.u32_to_i64(d["dip"])])
    words = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
    return docs, words, torch.full_like(words, int(dupfactor))


@traced("oni:flow.run")
def run_flow(cols: dict, K: int = 20, sweeps: int = 200, tol: float = 1.0, maxresults: int = 3000,
             alpha: float | None = None, beta: float | None = None, seed: int = 0x0D15EA5E, chunk_len: int = 0,
             device="cpu", comm: Comm | None = None, feedback: dict | None = None, dupfactor: int = 1000,
             row_offset: int = 0, eval_every: int = 0, burnin: int = 0, ckpt=None, log=None, ldac_dir: str | None = None,
             ldac_lag: int = 0, device_cols: dict | None = None, on_train=None) -> FlowResult:
    """Full suspicious-connects for one (rank-local shard of a) day of flows. ``device_cols``:
    the day's :data:`DEVICE_COLS` already on the device (e.g. from io.staging.Prefetcher, which
    uploaded them while the previous day computed); ``cols`` still supplies the host rows.
    ``on_train``: see :func:`common.build_and_train`."""
    timer = StageTimer(device)
    if device_cols is None:
        cols, feedback = with_ipv6_keys(cols, comm, (feedback,)) if feedback else (with_ipv6_keys(cols, comm), None)
    elif _needs_v6_keys(cols) or _needs_v6_keys(feedback):
        # prefetched device columns were uploaded from the host rows as they were: a day with IPv6
        # rows must be keyed (with its feedback, one shared dictionary) BEFORE pinning, as the
        # multi-day loader does (pipeline.daily.load_host_day)
        raise ValueError("run_flow(device_cols=...): IPv6 rows must be keyed with with_ipv6_keys() before the "
                         "columns are pinned and uploaded (feedback rows too)")
    with timer.stage("h2d"):
        d = dict(device_cols) if device_cols is not None else to_device(cols, device)
    with timer.stage("featurize"):
        cuts = compute_cuts(d, comm)
        sw, dw = wordify(d, cuts)
    with timer.stage("vocab"):
        n = d["sip"].numel()
        doc_keys = ops.widen_pair(d["sip"], d["dip"])
        word_keys = ops.widen_pair(sw, dw)
        weights = None
        fb = feedback_tokens(feedback, cuts, device, dupfactor)
        if fb is not None:
            # every rank reads the same feedback file: all of them carry token weights (the
            # routing exchanges the same columns everywhere), only rank 0 adds the tokens
            weights = torch.ones_like(word_keys, dtype=torch.int32)
            if common.feedback_here(comm):
                weights = torch.cat([weights, fb[2].to(torch.int32)])
                doc_keys = torch.cat([doc_keys, fb[0]])
                word_keys = torch.cat([word_keys, fb[1]])
        # flow words are 29-bit keys (spec.flow_word_str layout)
        vocab, wids = common.encode_words(word_keys, comm, key_bits=32)
    run = common.build_and_train(doc_keys, None, weights, vocab, K, alpha, beta, seed, sweeps, chunk_len, comm,
                                 eval_every=eval_every, burnin=burnin, ckpt=ckpt, log=log, timer=timer, ldac_dir=ldac_dir,
                                 ldac_lag=ldac_lag, word_ids=wids, n_event0=n, on_train=on_train)

    # ---- scoring --------------------------------------------------------------------------------
    hist = torch.zeros(2048, dtype=torch.int32, device=d["sip"].device)
    plan = None
    if run.route is not None:
        # data parallel: pairs are scored where their θ rows live, token scores come back (X05')
        with timer.stage("score_prep"):
            ts = common.owner_token_scores(run, comm)
        with timer.stage("score"):
            score, s1, s2 = common.owner_event_scores(ts, n, 2, tol, hist, want_parts=True)
            rows, scs = common.top_n(score, tol, maxresults, comm, row_offset, hist=hist)
    else:
        with timer.stage("score_prep"):
            dkeys, theta = common.gather_theta(run, comm)
            phi = run.model.phi()
            if run.pairs is not None and not common.SCORE_TILES:
                plan = common.plan_from_pairs(run.pairs, n, 2)  # the corpus pair build holds the plan
            else:
                plan = common.event_score_plan(run, dkeys, vocab, [doc_keys[:n], doc_keys[n: 2 * n]], wids[: 2 * n],
                                               [word_keys[:n], word_keys[n: 2 * n]], comm)
        with timer.stage("score"):
            score, s1, s2 = common.plan_score(theta, phi, plan, tol, hist=hist, want_parts=True, run=run)
            rows, scs, rpos = common.top_n(score, tol, maxresults, comm, row_offset, hist=hist, order=plan.order,
                                           return_pos=True)
    t = timer.summary()
    t.update(run.timings)
    t["records_scored"] = n
    # per-result parts (rows are global ids; each rank contributes its own rows)
    loc = rows - row_offset
    mine = (loc >= 0) & (loc < n)
    li = loc[mine]
    pi = rpos[mine] if plan is not None else li  # positions of the result events in score order
    if s1 is not None and not pi.is_cuda and s1.is_cuda:
        # host result positions (world 1): one upload of both index sets, one copy back
        ix = torch.stack([pi, li]).to(s1.device, non_blocking=True)
        got = torch.stack([s1[ix[0]], s2[ix[0]], sw[ix[1]].view(torch.float32),
                           dw[ix[1]].view(torch.float32)]).cpu()
        parts = got[:2].T.contiguous()
        wparts = got[2:].T.contiguous().view(torch.int32)
    else:
        parts = torch.stack([s1[pi], s2[pi]], 1) if s1 is not None else torch.zeros(0, 2)
        wparts = torch.stack([sw[li], dw[li]], 1)
    if comm is not None and comm.dist:
        # one all-gather of (global row id, both parts' f32 bits, both words) for this rank's rows
        packed = torch.cat([rows[mine].to(torch.int64).view(-1, 1), parts.to(torch.float32).view(torch.int32).to(torch.int64),
                            wparts.to(torch.int64) & common.U32MASK], 1)
        allp = torch.cat(comm.allgather_var(packed.contiguous())).cpu()
        order = common.rows_in_order(allp[:, 0], rows.cpu())
        allp = allp[order]
        parts = allp[:, 1:3].to(torch.int32).view(torch.float32)
        wparts = allp[:, 3:5].to(torch.int32)
    stats = run.corpus.stats()
    stats.update({"n_flows": n, "loglik": run.model.likelihoods[-1][1] if run.model.likelihoods else None})
    return FlowResult(rows=rows.cpu().numpy(), scores=scs.cpu().numpy(), src_scores=parts[:, 0].cpu().numpy(),
                      dst_scores=parts[:, 1].cpu().numpy(), src_words=wparts[:, 0].cpu().numpy().view(np.uint32),
                      dst_words=wparts[:, 1].cpu().numpy().view(np.uint32), cuts=cuts, timings=t, stats=stats,
                      lda=run)
