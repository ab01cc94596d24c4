"""Collapsed-Gibbs LDA engine (device-resident, data-parallel over documents).

The MI355X replacement of oni-lda-c ``lda est``: instead of
variational EM over an on-disk corpus shipped to MPI ranks, the corpus (SELL layout, see
:mod:`oni355.models.corpus`) and all count matrices live in HBM; one sweep is

    copy long-doc rows → k_gibbs (sample every token) → [RCCL all-reduce of Δn_wk ‖ Δn_k] → k_apply

Outputs mirror lda-c (``final.beta`` = log φ, ``final.gamma`` = n_dk + α, ``final.other``,
``likelihood.dat``, ``word-assignments.dat``; see :mod:`oni355.io.ldac`).

Determinism contract: every z is a pure function of (data, seed, sweep) — the same for 1 or N
GPUs, any chunk packing, and across checkpoint/resume (tests/test_gibbs*.py).
"""
from __future__ import annotations

import gc
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..ref import spec
from ..utils.obs import traced
from ..utils import fault
from .corpus import Corpus, canonical_tokens


NK_REP = 32
# the word-side Dirichlet prior β when none is given (default_beta): 0.1 from BETA_WIDE_MIN_K topics,
# 0.01 below
BETA_WIDE_MIN_K = 100


def default_beta(K: int) -> float:
    """β when the caller gives none: 0.1 for K ≥ BETA_WIDE_MIN_K (the config-5 models), else 0.01.
    Round-6 A/B (docs/performance.md, profiles/r6/beta/): at K = 100 β = 0.1 lifts top-3000 recall
    on the config-5 flow share 0.35 → 0.985 and on the 62.5M-flow day 0.405 → 0.455 at the same day
    time; below, the A/Bs were mixed (proxy quiet-client plants 0.88 → 1.0, DNS own-client plants
    0.66 → 0.62) and on small days with many topics (6000 DNS events, K = 50) Vβ outweighs a topic's
    tokens and recall collapses -- so the K = 20 / 50 models keep 0.01."""
    return 0.1 if K >= BETA_WIDE_MIN_K else 0.01
POLL_GIVE_UP_SWEEP = 40  # auto count mode: last sweep that may still start a far-off switch
# largest global token count a model takes: every int32 count (n_wk, n_k, n_dk, Δ) is ≤ the token
# count, and the Δn_k replicas hold partial sums of it
INT32_COUNT_MAX = 2**31 - 1
# X01 payload packing pays only once the all-reduce is bandwidth-bound (see GibbsLDA._x01_wanted)
X01_PACK_MIN_BYTES = 4 << 20
# sweep kernels (-> oni_gibbs_launch variant argument): every one draws the same topics bit for bit
MH_ALIAS_MAX_BYTES = 128e6  # word alias records above this size (half the MALL) use the CDF proposal
SAMPLERS = {"generic": 0, "lds": 2, "x1": 3, "mh": ops.SAMPLER_MH}


# "auto" runs the MH sampler from this many topics (env ONI_MH_AUTO_MIN_K), after the dense burn-in
# of mh_burn_for(): at K = 100 its sweep is 3.2 vs 6.6 ms on the config-5 flow model, and started
# from 20 dense sweeps its chain holds the dense chain's log-likelihood (+0.1 % at sweep 200; from a
# random start it burns in slowly, −3 %). Config-5 day 2.110 → 1.444 s at recall 0.99 / 1.0 / 0.865
# (dense 0.995 / 1.0 / 0.845; profiles/r4/combined_day_config5_share_125M_{dense,mh_burn20}.json).
# At K = 50 the dense kernel is the faster one.
MH_AUTO_MIN_K = int(os.environ.get("ONI_MH_AUTO_MIN_K", "100"))


def sampler_for(K: int, sampler: str | None = None) -> str:
    """The sweep kernel family a K-topic model runs: ``sampler`` or ONI_SAMPLER (default "auto");
    "auto" resolves to "mh" for K ≥ MH_AUTO_MIN_K and to "dense" (k_gibbs_x1 / k_gibbs_ldsg) below.
    The corpus must be built for its tiling (:func:`tiling_for`)."""
    s = sampler if sampler is not None else os.environ.get("ONI_SAMPLER", "auto")
    if s == "auto":
        # the lagged X01 (ONI_X01_LAG) runs the dense samplers only
        return "mh" if K >= MH_AUTO_MIN_K and not x01_lag_on() else "dense"
    return s


def x01_lag_on() -> bool:
    """ONI_X01_LAG=1: the X01 all-reduce of sweep s is issued asynchronously and runs beside the
    sampler of sweep s + 1 (GibbsLDA._x01_start): from sweep ONI_X01_LAG_FROM every sweep samples
    its word side against the global counts one sweep older than its doc rows -- the same rule on
    any number of GPUs."""
    return os.environ.get("ONI_X01_LAG", "0") == "1"


def mh_burn_for(sweeps: int) -> int:
    """Dense sweeps an MH model runs before its own (env ONI_MH_BURN, default 20): the pipeline
    samples them with the exact dense kernel on a second corpus of the dense tiling and hands the
    chain over through its canonical z (:meth:`GibbsLDA.load_canonical_z`). From a random start
    the MH chain burns in slowly on large models (−3 % log-likelihood at sweep 200 on the
    125M-token flow model); started from the dense chain's state it holds the dense chain's
    equilibrium (+0.01 % after 40 dense sweeps, +0.1 % after 20, −0.45 % after 10:
    profiles/r4/mh_quality_gpu_62.5M_k100_burn*.json)."""
    return max(0, min(int(os.environ.get("ONI_MH_BURN", "20")), int(sweeps)))


def tiling_for(K: int, sampler: str | None = None) -> tuple[int, int]:
    return ops.choose_tiling(K, "mh" if sampler_for(K, sampler) == "mh" else None)


@dataclass
class GibbsConfig:
    K: int = 20
    alpha: float | None = None  # default 50/K (Griffiths & Steyvers)
    beta: float | None = None  # None: default_beta(K)
    seed: int = 0x0D15EA5E
    use_graph: bool = True
    # n_wk bookkeeping: "auto" (default: "recount" while most topics still move, then "delta"),
    # "dual" (changed topics mirrored into a word-sorted z copy, streaming recount), "delta"
    # (changed-slot masks + word-sorted delta recount: cost ∝ changed tokens), "recount" (full
    # gathered recount: constant cost) | "atomic" (per-token Δ atomics)
    # "wdelta" (changed tokens set a bit in a word-sorted bitmap + keep (old, new) topics in
    # word-sorted order: the recount touches only changed tokens, no slot indirection).
    # ONI_COUNT_MODE overrides the default.
    count_mode: str = field(default_factory=lambda: os.environ.get("ONI_COUNT_MODE", "auto"))
    # "auto": switch to the delta recount once the all-reduced fraction of tokens that changed
    # topic in a sweep falls below auto_threshold (measured on device, read two sweeps late so the
    # host never stalls the stream); auto_switch > 0 instead fixes the first delta sweep (tests)
    auto_switch: int = 0
    # 0.19: the wdelta sweep beats the full recount below ~15-25 % changed tokens since its records
    # carry the word row (default flow day 58.6 ms at 0.12, 58.0-58.2 at 0.16 / 0.19 / 0.22 / 0.30;
    # DNS 26.1 ms at 0.30, 25.2-25.3 below; profiles/r5/auto_threshold/)
    auto_threshold: float = field(default_factory=lambda: float(os.environ.get("ONI_AUTO_THRESHOLD", "0.19")))
    # the delta bookkeeping auto mode switches to: "wdelta" (word-sorted change bitmap) | "delta"
    auto_delta: str = field(default_factory=lambda: os.environ.get("ONI_AUTO_DELTA", "wdelta"))
    # debug: verify count invariants after every sweep() call (ONI_CHECK_INVARIANTS=1)
    check_invariants: bool = field(default_factory=lambda: os.environ.get("ONI_CHECK_INVARIANTS", "0") == "1")
    # cheap numerical health check after every sweep() call (ONI_HEALTH_CHECK=0 disables)
    health_check: bool = field(default_factory=lambda: os.environ.get("ONI_HEALTH_CHECK", "1") != "0")
    # sweep kernel: "auto" (default: "dense"; "mh" for K ≥ MH_AUTO_MIN_K = 100), "dense" ("x1" for
    # K ≤ 32, "lds" above), "x1" the one-lane register sampler k_gibbs_x1, "lds" the multi-lane
    # LDS-count sampler k_gibbs_ldsg, "generic" k_gibbs (any unit width; the fallback when n + α is
    # not exact in f32) -- these are bitwise identical to each other and to spec.gibbs_pass --
    # and "mh" the Metropolis-Hastings sampler k_gibbs_mh (its own chain, spec.gibbs_pass_mh).
    # ONI_SAMPLER overrides the default.
    sampler: str = field(default_factory=lambda: os.environ.get("ONI_SAMPLER", "auto"))
    # posterior averaging: θ and φ are estimated from the counts of the last ``post_samples``
    # samples taken every ``post_every`` sweeps (ending at the last sweep) instead of the final
    # sample alone. A word seen once sits in ONE topic in any single sample, so its φ row -- and
    # the score of its event -- follows that one draw: a rare word sampled into a minor topic of
    # its document scores as if it were an anomaly. The averaged counts give it its posterior
    # topic mix, as lda-c's variational β / γ do. 1 = the final sample only.
    # Default: every sweep of the last quarter of the chain, at most 50 (sweeps 151-200 of a
    # 200-sweep day). With post_every = 1 the sample sums are added inside the captured sweep
    # graphs (three integer adds per sweep), so the averaging costs no eager launches.
    post_samples: int = field(default_factory=lambda: int(os.environ.get("ONI_POST_SAMPLES", "50")))
    post_every: int = field(default_factory=lambda: int(os.environ.get("ONI_POST_EVERY", "1")))
    # initial topics: "random" (Philox stream 0 per token) or "word" (every token of a word in the
    # word's hashed topic, independent of the seed: chains of different seeds start together)
    init: str = field(default_factory=lambda: os.environ.get("ONI_INIT", "random"))
    # lagged X01 (ONI_X01_LAG, x01_lag_on): the sweep's Δ all-reduce overlaps the next sweep
    x01_lag: bool = field(default_factory=x01_lag_on)

    def resolved_alpha(self) -> float:
        return float(self.alpha) if self.alpha is not None else 50.0 / self.K

    def resolved_beta(self) -> float:
        return float(self.beta) if self.beta is not None else default_beta(self.K)


def _alpha_in_row_exact(alpha: float, max_doc_len: int) -> bool:
    """May the LDS samplers keep n + α (f32) in their rows? Only if every n + α with
    0 ≤ n ≤ max_doc_len is exact in f32, so the rows' ±1 updates reproduce fl(n) + α bit for bit."""
    a = float(np.float32(alpha))
    if not (a > 0 and math.isfinite(a)):
        return False
    f = 0
    while f <= 23 and a * (1 << f) != math.floor(a * (1 << f)):
        f += 1
    return f <= 23 and max_doc_len + math.ceil(a) < (1 << (24 - f))


_CAPTURE_STREAMS: dict = {}


def _capture_stream(device) -> "torch.cuda.Stream":
    """One side stream per device for every graph capture: a fresh stream per capture cost ~1.5 ms
    of host time at its first cross-stream wait (two captures per day)."""
    key = str(device)
    if key not in _CAPTURE_STREAMS:
        _CAPTURE_STREAMS[key] = torch.cuda.Stream(device)
    return _CAPTURE_STREAMS[key]


class GibbsLDA:
    """Device state + sweep loop. ``comm`` (oni355.parallel.comm.Comm) enables data parallelism."""

    def __init__(self, corpus: Corpus, cfg: GibbsConfig, comm=None, V_global: int | None = None):
        self.c = corpus
        self.cfg = cfg
        self.comm = comm
        self.K = cfg.K
        self.G, self.KP = tiling_for(cfg.K, cfg.sampler)
        if corpus.G != self.G:
            raise ValueError(f"corpus built for G={corpus.G}, K={cfg.K} needs G={self.G}")
        self.KS = self.G * self.KP
        self.alpha = cfg.resolved_alpha()
        self.beta = cfg.resolved_beta()
        self.V = int(V_global if V_global is not None else corpus.V)
        self.vbeta = float(np.float32(self.V * self.beta))
        dev = corpus.tok_word.device
        self.device = dev
        D, V, KS = corpus.D, self.V, self.KS
        i32 = torch.int32
        # count tables and z are zeroed by initialize() / load_canonical_z() before any use
        self.tok_z = torch.empty(corpus.sell_slots, dtype=torch.uint8, device=dev)
        self.ndk = [torch.empty(max(D, 1), KS, dtype=i32, device=dev) for _ in range(2)]
        self.nwk = torch.empty(V, KS, dtype=i32, device=dev)
        self.nk = [torch.empty(KS, dtype=i32, device=dev) for _ in range(2)]
        # Δn_k in NK_REP replicas (block b adds into b % NK_REP): the per-block topic totals
        # would otherwise queue thousands of same-address atomics on KS words
        self._aux_off = V * KS + NK_REP * KS
        # heavy documents cut across ranks (pipeline.common.SplitPlan): their per-rank Δn_dk rows
        # ride at the end of the X01 buffer ([V·KS | NK_REP·KS | DN_AUX | n_split·KS])
        self._split = None
        sp = corpus.split
        if sp is not None and comm is not None and comm.dist and int(sp["n_split"]) > 0:
            pr, qr = sp["piece_rows"].to(dev), sp["prim_rows"].to(dev)
            pj, qj = sp["piece_j"].to(dev), sp["prim_j"].to(dev)
            self._split = dict(n=int(sp["n_split"]), piece_rows=pr, piece_j=pj, all_rows=torch.cat([pr, qr]),
                               all_j=torch.cat([pj, qj]))
        self._split_off = self._aux_off + ops.DN_AUX
        n_split = self._split["n"] if self._split is not None else 0
        self.dn = [torch.empty(self._split_off + n_split * KS, dtype=i32, device=dev) for _ in range(2)]
        self.q = torch.zeros(V, KS, dtype=torch.float32, device=dev)
        # token-exclusion constants of the word side (A, B per topic; written with q by k_apply)
        self.qfix = torch.zeros(2, KS, dtype=torch.float32, device=dev)
        self.sweep_ctr = torch.zeros(1, dtype=i32, device=dev)
        if cfg.count_mode not in ("auto", "dual", "delta", "recount", "atomic", "wdelta"):
            raise ValueError(f"unknown count_mode {cfg.count_mode}")
        self.auto = cfg.count_mode == "auto"
        # auto: full recount while most topics still move, then the delta mode named by auto_delta
        auto_delta = {"wdelta": 4, "delta": 2}[cfg.auto_delta]
        self.mode = {"recount": 0, "atomic": 1, "delta": 2, "dual": 3, "wdelta": 4, "auto": auto_delta}[cfg.count_mode]
        # the auxiliary topic state of self.mode (z_prev for 2, word-sorted z_w for 4) matches tok_z
        self._aux_synced = False
        self._delta_on = False
        self._force_mode = None
        self._chg_q: list = []    # (sweep index, host buffer, event) of pending change-count copies
        self._poll_off = False
        self.T_global = corpus.T
        self.change_log: list[tuple[int, float]] = []
        # auto's early (high change rate) sweeps: "recount" (0, default) rebuilds n_wk by the
        # gathered recount; "dual" (3) keeps a word-sorted z copy current for changed tokens so the
        # recount streams it (1 B per token) -- measured slower on the 12.5M-flow day (0.2673 ->
        # 0.2718 ms/sweep: the sampler's scattered byte stores cost more than the gather saves).
        # ONI_AUTO_EARLY overrides.
        early = os.environ.get("ONI_AUTO_EARLY", "recount")
        if early not in ("dual", "recount"):
            raise ValueError(f"unknown ONI_AUTO_EARLY {early}")
        self.early = 3 if (self.auto and self.mode == 4 and early == "dual") else 0
        self._zw_synced = False  # z_w == tok_z in word-sorted order
        if self.mode == 3 or self.early == 3:
            self.z_w = torch.empty(max(corpus.T, 1), dtype=torch.uint8, device=dev)  # synced before use
        if self.mode == 4:
            # word-sorted change bitmap (+ slack word) and per-position records: (old | new << 8) of
            # each changed token (only read where a bit is set, so never synced with tok_z) next to
            # the position's word row in its recount block (written once here)
            self.wbits = torch.empty((corpus.T + 31) // 32 + 1, dtype=torch.int32, device=dev)  # _sync_aux_z zeroes
            self.zz_w = ops.wdelta_records(corpus.wsorted)
        if self.mode == 2:
            self.tok_zprev = torch.zeros_like(self.tok_z)
            self.chg_mask = torch.zeros(max(corpus.sell_slots // corpus.S, 1), dtype=torch.int64, device=dev)
        if cfg.sampler not in SAMPLERS and cfg.sampler not in ("auto", "dense"):
            raise ValueError(f"unknown sampler {cfg.sampler}")
        samp = sampler_for(cfg.K, cfg.sampler)
        self.mh = samp == "mh"
        if samp == "dense":
            self.qpf = SAMPLERS["x1"] if self.G == 1 else SAMPLERS["lds"]
        elif self.mh:
            self.qpf = SAMPLERS["mh"]
            self._setup_mh()
        else:
            self.qpf = SAMPLERS[samp]
            if (self.qpf == SAMPLERS["x1"]) != (self.G == 1) and self.qpf != SAMPLERS["generic"]:
                raise ValueError(f"sampler {cfg.sampler} does not run {self.G}-lane units (K = {cfg.K})")
        # the specialised kernels keep n + α as f32 in their count rows: exact only when every
        # n + α of this corpus is (one device read of the longest document); else generic
        self._air = False
        self._guard = None
        if self.qpf not in (SAMPLERS["generic"], SAMPLERS["mh"]):
            self._air = _alpha_in_row_exact(self.alpha, corpus.max_doc_len())
            if not self._air:
                # a document longer than the exact range: the row kernels may still run on every
                # sweep whose counts stay inside it -- decided per sweep on the device
                self._guard = self._make_guard()
                self._air = self._guard is not None
            if not self._air:
                self.qpf = SAMPLERS["generic"]
        # the Markov chain this model runs (checkpoint identity): the dense kernels are bitwise
        # one chain; MH is another, and its pipeline sets the dense burn-in it starts from
        self.chain = {"sampler": "mh" if self.mh else "dense", "mh_burn": 0}
        if self.mh:
            self.chain["mh_word"] = self.mh_word
        # lagged X01 (cfg.x01_lag): the word side of sweep s samples against the global counts
        # through sweep s − 2 (one sweep behind the doc rows) while Δ_{s−1} is reduced beside the
        # sampler. tok_zlag = each token's topic in those counts (the word-side exclusion is taken
        # there, spec.gibbs_pass); x01_red = the reduced Δ of the previous sweep that the sweep's
        # apply adds; its count mode decides absolute / delta (_pend_abs). Every sweep() call
        # ends in a drain (_lag_drain): the counts are current between calls.
        self.lag = bool(cfg.x01_lag)
        if self.lag:
            if self.mh:
                raise ValueError("the lagged X01 (ONI_X01_LAG) runs the dense samplers only")
            self.chain["x01_lag"] = 1
            self.tok_zlag = torch.empty_like(self.tok_z)
        self._pend_abs = False
        self._lag_base = 0
        # the lag starts at sweep ONI_X01_LAG_FROM (default 20: past the burn-in's high-change
        # sweeps -- the auto count mode switches at 16-20 on the measured days -- so one sweep of
        # staleness costs the chain little; from a random start it slows the burn-in:
        # docs/performance.md). A fixed sweep, so a resumed run starts it where the original did
        self._lag_live = False
        self._lag_from = int(os.environ.get("ONI_X01_LAG_FROM", "20"))
        self.a = 0  # ndk parity
        self.b = 0  # delta-buffer parity
        self.cn = 0  # nk parity
        self.sweeps_done = 0
        self.likelihoods: list[tuple[int, float]] = []
        self._graph = None
        self._graphs: dict = {}
        self._eager_lead_done = False  # the eager pair that hides a model's first capture (_sweep_n)
        self._watchdog = fault.Watchdog.from_env()
        self.timings = {"allreduce_calls": 0}
        self._ar_events: list = []
        self._capturing = False
        self._last_inplace = False  # the last executed sweep applied in place (Δ heads untouched)
        self._corrupted = False
        self._tail_cache = None  # (sweeps_done, device tail sums, host copy): see _tail()
        self._x01 = None
        if comm is not None and comm.dist and self.KS % 2 == 0 and self._x01_wanted():
            self._setup_x01()
        if self.lag:
            self.x01_red = torch.zeros_like(self.dn[0])
        # one rank (no process group, or a 1-rank group whose all-reduce is the identity): the count
        # passes add Δn_wk straight into n_wk and k_apply refreshes q from it (2 of its 5 passes
        # over V·KS fewer); ONI_APPLY_INPLACE=0 keeps the Δ buffer
        self._inplace_ok = ((comm is None or not comm.live and self._x01 is None)
                            and self._split is None and not self.lag
                            and os.environ.get("ONI_APPLY_INPLACE", "1") != "0")
        # chunk starts (doc-local token positions) are multiples of the chunk length L, pieces of
        # split documents included: with L % 4 == 0 every chunk starts a Philox 4-token group
        self._pos_aligned = int(self.c.L) % 4 == 0
        self._avg = None          # posterior-averaging accumulators (plan_average)
        self._acc = False         # sweeps add their counts to the accumulators (inside graphs too)
        self._avg_at: list = []   # sweep counts at which a sample is added
        self._avg_cache = None    # (θ, φ) of the completed average

    def _make_guard(self):
        """Device exactness guard (k_exact_guard) for a corpus with documents past the range in
        which n + α is exact in f32: (rows to check, count limit, flag). A chunk moves its row by at
        most its length L from the sweep-start counts, so the row kernels are exact for a sweep iff
        every sweep-start count of a row that can pass limit = N_safe − L is ≤ limit; only rows
        longer than that can (split documents: their global counts). None when no guard fits, or
        ONI_EXACT_GUARD=0 (the generic kernel on every sweep, as before)."""
        if os.environ.get("ONI_EXACT_GUARD", "1") == "0" or self.device.type != "cuda" and not os.environ.get(
                "ONI_EXACT_GUARD_CPU"):
            return None
        lo, hi = 0, 1 << 25
        while lo < hi:  # largest n with every count ≤ n exact
            mid = (lo + hi + 1) // 2
            lo, hi = (mid, hi) if _alpha_in_row_exact(self.alpha, mid) else (lo, mid - 1)
        c = self.c
        Lmax = int(c.chunk_len.max()) if c.chunk_len.numel() else int(c.L)
        limit = lo - max(Lmax, int(c.L))
        if os.environ.get("ONI_EXACT_GUARD_LIMIT"):  # tests: force the generic side
            limit = min(limit, int(os.environ["ONI_EXACT_GUARD_LIMIT"]))
        if limit < 0:
            return None
        lens = c.doc_lengths().to(torch.int64)
        risky = torch.nonzero(lens > limit).flatten()
        if c.split is not None and int(c.split["max_count"]) > limit:
            sp = c.split
            risky = torch.unique(torch.cat([risky.to(self.device), sp["piece_rows"].to(self.device).to(torch.int64),
                                            sp["prim_rows"].to(self.device).to(torch.int64)]))
        return dict(rows=risky.to(torch.int32).to(self.device), limit=int(limit),
                    flag=torch.ones(1, dtype=torch.int32, device=self.device))

    def _setup_mh(self) -> None:
        """MH sampler state: per-sweep proposal tables (every word's level-1 CDF row; alias rows of
        the documents spread over several chunks, which propose from their sweep-start row) and
        every chunk's row in the doc table."""
        c = self.c
        if c.L > spec.MH_MAX_CHUNK or (c.chunk_len.numel() and int(c.chunk_len.max()) > spec.MH_MAX_CHUNK):
            raise ValueError(f"the MH sampler needs chunks of at most {spec.MH_MAX_CHUNK} tokens (corpus L = {c.L})")
        dev = self.device
        live = c.chunk_doc >= 0
        multi = live & (c.chunk_multi != 0)
        rows = torch.unique(c.chunk_doc[multi].to(torch.int64))
        self.mh_rows = rows.to(torch.int32)
        dslot = torch.full_like(c.chunk_doc, -1)
        if rows.numel():
            dslot[multi] = torch.searchsorted(rows, c.chunk_doc[multi].to(torch.int64)).to(torch.int32)
        self.chunk_dslot = dslot
        # word proposal ∝ q[w, ·] (ONI_MH_WORD, default "auto"): "alias" -- every word's alias row as
        # 16-B records built per sweep (one gather per proposal; the build writes V·K·16 B), or "cdf"
        # -- a 64-B row of bucket prefix sums per word (a streaming pass over q) with the bucket's q
        # values as the second level (two gathers and ~60 more VALU per token). "auto" takes the CDF
        # when 3·V·K > 2·T (global tokens): measured at K = 100 the record build costs ~10 ps per
        # cell and the CDF draw ~6 ps per token more (profiles/r5/) -- or when the records
        # (V·K·16 B) outgrow half of the 256 MB MALL, where their gathers miss: at V = 349k,
        # T = 125M the CDF ran 4.38 against the records' 4.62 ms/sweep
        # (profiles/r5/bench_k100_realistic_62.5M_{alias,cdf}.json).
        T_all = torch.tensor([float(c.T)], dtype=torch.float64)
        if self.comm is not None and self.comm.dist:
            T_all = self.comm.allreduce_(T_all.to(self.comm.device)).cpu()
        kind = os.environ.get("ONI_MH_WORD", "auto")
        if kind == "auto":
            kind = ("cdf" if 3.0 * self.V * self.K > 2.0 * float(T_all[0]) or 16.0 * self.V * self.K > MH_ALIAS_MAX_BYTES
                    else "alias")
        if kind not in ("alias", "cdf"):
            raise ValueError(f"unknown ONI_MH_WORD {kind}")
        self.mh_word = kind
        self.walias = self.wsum = self.wcdf = None
        if kind == "cdf":
            self.wcdf = torch.zeros(self.V, spec.MH_CDF_BUCKETS, dtype=torch.float32, device=dev)
        else:
            self.walias = torch.zeros(self.V, self.K, 4, dtype=torch.int32, device=dev)  # 16-B records
            self.wsum = torch.zeros(self.V, dtype=torch.float32, device=dev)
        self.dalias = torch.zeros(max(int(rows.numel()), 1), self.K, dtype=torch.int32, device=dev)
        self.mh_g = torch.zeros(self.KS, dtype=torch.float32, device=dev)
        # one word move + two doc moves per token: with one doc move the chain plateaus 2.6 % lower
        # in log-likelihood on the 12.5M-flow day (rare words' word tables mostly propose the
        # token's own topic); two match the dense chain at the same chunk length
        # (profiles/r4/mh_quality_gpu_*.json)
        self.mh_doc_moves = int(os.environ.get("ONI_MH_DOC_MOVES", "2"))
        self.mh_lmax = max(1, min(int(c.L), spec.MH_MAX_CHUNK))

    def mh_build_tables(self) -> None:
        """The sweep's MH proposal tables from the snapshot (q and the topic totals nk[cn] the last
        apply wrote, the sweep-start doc rows ndk[a])."""
        ops.mh_tables(self.q, self.nk[self.cn], self.ndk[self.a], self.mh_rows, self.K, self.alpha, self.vbeta,
                      self.dalias, self.mh_g, walias=self.walias, wsum=self.wsum, wcdf=self.wcdf)

    def mh_state(self) -> dict:
        return dict(walias=self.walias, wsum=self.wsum, wcdf=self.wcdf, dalias=self.dalias, mh_g=self.mh_g,
                    chunk_dslot=self.chunk_dslot, mh_lmax=self.mh_lmax)

    def _x01_wanted(self) -> bool:
        """``ONI_X01_PACK``: "1" always packs, "0" never, "auto" (default) packs when the dense Δ
        buffer is at least ``ONI_X01_PACK_MIN_BYTES`` (default 4 MiB). Below that the all-reduce
        is latency-bound (a 0.46 MB flow-day buffer costs about the same as half of it) and the
        pack + unpack kernels would be two extra graph nodes per sweep for nothing."""
        mode = os.environ.get("ONI_X01_PACK", "auto")
        if mode in ("0", "1"):
            return mode == "1"
        min_bytes = int(os.environ.get("ONI_X01_PACK_MIN_BYTES", str(X01_PACK_MIN_BYTES)))
        return self.dn[0].numel() * self.dn[0].element_size() >= min_bytes

    def _setup_x01(self) -> None:
        """Packed X01 payload (csrc/kernels/x01.hip). A word's per-rank value (an absolute local
        count in recount sweeps, a delta otherwise) is bounded by its local token count c_{w,r}, so
        words with max_r c_{w,r} ≤ O8 = ⌊127 / W⌋ travel as four offset bytes per int32 word, words
        up to O = ⌊32767 / W⌋ as two offset 16-bit halves, and the ring sum stays exact; the rest
        stays int32. A realistic vocabulary is mostly rare words: 13.6 MB → ~3.4 MB per sweep at
        V = 170k, K = 20 (dense → 8-bit)."""
        W = self.comm.world
        O = 32767 // W
        O8 = 127 // W
        if os.environ.get("ONI_X01_LIGHT_MAX"):  # tests: force a tiny/light/heavy mix on small days
            O = min(O, int(os.environ["ONI_X01_LIGHT_MAX"]))
        if os.environ.get("ONI_X01_TINY_MAX"):
            O8 = min(O8, int(os.environ["ONI_X01_TINY_MAX"]))
        O8 = min(O8, O)
        V, KS = self.V, self.KS
        dev = self.device
        cnt = torch.zeros(V, dtype=torch.int64, device=dev)
        if self.c.T:  # wsorted is sorted: run lengths by binary search, no contended histogram
            ws = self.c.wsorted.to(torch.int64)
            edges = torch.searchsorted(ws, torch.arange(V + 1, dtype=torch.int64, device=dev))
            cnt += edges[1:] - edges[:-1]
        self.comm.allreduce_(cnt, op="max")
        if KS % 4:
            O8 = -1  # four counts per word need KS % 4 == 0 (always true for choose_tiling)
        tiny = torch.nonzero(cnt <= O8).flatten().to(torch.int32)
        light = torch.nonzero((cnt > O8) & (cnt <= O)).flatten().to(torch.int32)
        heavy = torch.nonzero(cnt > O).flatten().to(torch.int32)
        tail_off, tail_len = V * KS, self.dn[0].numel() - V * KS
        n = ops.x01_packed_len(tiny.numel(), light.numel(), heavy.numel(), KS, tail_len)
        if n >= self.dn[0].numel():
            return
        self._x01 = dict(tiny=tiny.contiguous(), light=light.contiguous(), heavy=heavy.contiguous(), O8=max(O8, 0),
                         O=O, WO8=W * max(O8, 0), WO=W * O, tail_off=tail_off, tail_len=tail_len,
                         buf=torch.zeros(n, dtype=torch.int32, device=dev))

    # ---------------------------------------------------------------------------------------------
    def _state(self, init: bool) -> dict:
        c = self.c
        # the sampler reads chunk_pos0 only as the Philox position: split pieces use global ones
        st = dict(tok_word=c.tok_word, tok_z=self.tok_z, slice_off=c.slice_off, slice_len=c.slice_len,
                  chunk_doc=c.chunk_doc, chunk_pos0=c.chunk_rng0 if c.chunk_rng0 is not None else c.chunk_pos0,
                  chunk_key=c.chunk_key, chunk_multi=c.chunk_multi, q=self.q, qfix=self.qfix)
        VK = self.V * self.KS
        if init:
            st.update(ndk_src=self.ndk[0], ndk_dst=self.ndk[0], dnwk=self.nwk, dnk=self.nk[0])
        else:
            d = self.dn[self.b]
            st.update(ndk_src=self.ndk[self.a], ndk_dst=self.ndk[1 - self.a], dnwk=d[:VK].view(self.V, self.KS),
                      dnk=d[VK:self._aux_off], chg_count=d[self._aux_off:self._aux_off + 1])
            if self._lag_live:
                st["tok_zlag"] = self.tok_zlag
        return st

    @traced("oni:lda.initialize")
    def initialize(self) -> None:
        """Random topic init (Philox stream 0), counts, first q table."""
        for t in (*self.ndk, self.nwk, *self.nk, *self.dn):
            t.zero_()
        self.tok_z.zero_()
        self.a = self.b = 0
        self.cn = 0
        # topics drawn without n_wk atomics, then n_wk rebuilt by the word-sorted recount (integer
        # counts: identical to the atomic build, without its same-address contention)
        st = self._state(True)
        if self.mh:
            st["mh_lmax"] = self.mh_lmax
        ops.gibbs_pass(st, self.G, self.KP, self.K, self.alpha, self.cfg.seed, True,
                       self.sweep_ctr, self.c.chunk_len, host_sweep=0, mode=0,
                       sampler=SAMPLERS["mh"] if self.mh else 0, word_init=self.cfg.init == "word")
        ops.recount(self.c.wsorted, self.c.wslot, self.tok_z, self.nwk, self.KS)
        self._split_sync_absolute(self.ndk[0])
        if self.comm is not None and self.comm.dist:
            self.comm.allreduce_(self.nwk)
            self.comm.allreduce_(self.nk[0])
        # one rank (a forced 1-rank group too): every token holds one topic, so Σ n_k = T (no device
        # read, no host sync behind the init kernels); DP: the global sum
        self.T_global = (int(self.nk[0][: self.K].sum()) if self.comm is not None and self.comm.live
                         else int(self.c.T))
        self._check_magnitude()
        self._delta_on = False
        self._chg_q = []
        self._poll_off = False
        self._sync_aux_z()
        self.sweeps_done = 0
        self._graph = None
        self._prime()

    def _check_magnitude(self) -> None:
        """Every count table (n_wk, n_k, n_dk, the Δ buffers) is int32 and bounded by the global
        token count: refuse a model whose tokens (feedback duplicates included) could wrap one,
        instead of sampling from garbage. The posterior-average sums are int64."""
        if self.T_global > INT32_COUNT_MAX or self.c.T > INT32_COUNT_MAX:
            raise ValueError(f"{self.T_global} global tokens: int32 count tables hold at most {INT32_COUNT_MAX} "
                             "(split the day or the source into several models)")

    # ---- split documents: one n_dk row per document across its pieces ---------------------------
    def _split_sync_absolute(self, ndk: torch.Tensor) -> None:
        """Rows of split documents := the sum of their pieces' counts over all ranks (after the
        init pass or a restore, when piece rows hold local counts and primary rows nothing)."""
        sp = self._split
        if sp is None:
            return
        tot = torch.zeros(sp["n"], self.KS, dtype=torch.int32, device=self.device)
        tot.index_add_(0, sp["piece_j"], ndk.index_select(0, sp["piece_rows"]))
        self.comm.allreduce_(tot)
        ndk.index_copy_(0, sp["all_rows"], tot.index_select(0, sp["all_j"]))

    def _split_delta(self, buf: torch.Tensor, src: torch.Tensor, dst: torch.Tensor) -> None:
        """X01 tail := this rank's Δn_dk of every split document (Σ over its pieces)."""
        sp = self._split
        reg = buf[self._split_off:].view(sp["n"], self.KS)
        reg.zero_()
        r = sp["piece_rows"]
        reg.index_add_(0, sp["piece_j"], dst.index_select(0, r) - src.index_select(0, r))

    def _split_apply(self, buf: torch.Tensor, src: torch.Tensor, dst: torch.Tensor) -> None:
        """After the all-reduce: every row of a split document := sweep-start row + global Δ."""
        sp = self._split
        reg = buf[self._split_off:].view(sp["n"], self.KS)
        r = sp["all_rows"]
        dst.index_copy_(0, r, src.index_select(0, r) + reg.index_select(0, sp["all_j"]))

    def _sweep_mode(self, sweep: int) -> int:
        """Count mode used by (1-based) sweep ``sweep``."""
        if self._force_mode is not None:
            return self._force_mode
        if self.auto:
            if self.cfg.auto_switch > 0:
                return self.early if sweep < self.cfg.auto_switch else self.mode
            return self.mode if self._delta_on else self.early
        return self.mode

    def _note_changes(self) -> None:
        """Queue an async copy of the last completed sweep's (all-reduced) changed-token count."""
        if not self.auto or self.cfg.auto_switch > 0 or self._delta_on or self._poll_off:
            return
        src = self.dn[1 - self.b][self._aux_off:self._aux_off + 1]
        sw = self.sweeps_done
        if self._lag_live:
            # the last sweep's count is still in flight: the reduced one of the sweep before
            src, sw = self.x01_red[self._aux_off:self._aux_off + 1], self.sweeps_done - 1
            if sw <= self._lag_base:
                return
        if self.device.type == "cuda":
            from ..io import staging
            buf = torch.empty(1, dtype=torch.int32, pin_memory=True)
            staging.push_to_host(src, buf)  # a kernel store: not queued behind a bulk H2D upload
            ev = torch.cuda.Event()
            ev.record()
        else:
            buf, ev = src.clone(), None
        self._chg_q.append((sw, buf, ev))

    def _decide_mode(self) -> None:
        """At even sweep counts, consume counts of sweeps ≤ now-2 (deterministic on every rank)."""
        if not self._chg_q or self.sweeps_done % 2:
            return
        latest = None
        while self._chg_q and self._chg_q[0][0] <= self.sweeps_done - 2:
            sw, buf, ev = self._chg_q.pop(0)
            if ev is not None:
                ev.synchronize()
            latest = (sw, int(buf[0]) / max(self.T_global, 1))
        if latest is not None:
            self.change_log.append(latest)
            if latest[1] < self.cfg.auto_threshold:
                self._delta_on = True
                self._chg_q.clear()
            elif latest[0] >= POLL_GIVE_UP_SWEEP and latest[1] > 2 * self.cfg.auto_threshold:
                # still far above the switch point this late (the DNS day holds at ~67 % changed
                # tokens): stop the per-pair-of-sweeps count read-back. Count modes all draw the
                # same chain, so this only trades a possible late switch for 100 fewer polls
                self._poll_off = True
                self._chg_q.clear()

    def _ensure_zw(self) -> None:
        """Word-sorted z copy := tok_z before a dual-mode (3) sweep (eager, never captured)."""
        if not self._zw_synced and self.c.T:
            self.z_w[: self.c.T] = self.tok_z[self.c.wslot.long()]
        self._zw_synced = True

    def _sync_aux_z(self) -> None:
        """Bring the auxiliary topic copies (z_prev / word-sorted z) in line with tok_z."""
        if self.mode == 2:
            self.tok_zprev.copy_(self.tok_z)
        elif self.mode == 3 and self.c.T:
            self.z_w[: self.c.T] = self.tok_z[self.c.wslot.long()]
        elif self.mode == 4:
            self.wbits.zero_()
        self._aux_synced = True

    def _keeps_aux(self, mode: int) -> bool:
        """Does a sweep in count mode ``mode`` leave self.mode's auxiliary topic state in sync?"""
        return mode == self.mode or self.mode == 4  # MODE 4's bitmap is empty between sweeps

    def _prime(self) -> None:
        # zero-delta apply: q from n_wk, nk[1] = nk[0]; leaves dn[0], dn[1] zero
        self._tail_cache = None
        self._zw_synced = False  # tok_z was (re)written outside the sweeps (init / restore)
        VK = self.V * self.KS
        self.dn[0].zero_()
        so = self._split_off
        ops.gibbs_apply(self.nwk, self.dn[0][:so], self.dn[1][:so], self.nk[self.cn], self.nk[1 - self.cn], self.q,
                        self.qfix, self.V,
                        self.K, self.KS, self.beta, self.vbeta, self.sweep_ctr, bump=False,
                        rows_copy=(self.ndk[self.a], self.ndk[1 - self.a], self.c.long_rows))
        self.cn = 1 - self.cn
        self.sweep_ctr.fill_(self.sweeps_done + 1)
        self._last_inplace = False  # dn[0] zeroed here, dn[1] by the apply
        if self.lag:
            # the counts are current: the next sweep's word side counts every token at tok_z, and
            # the Δ it reduces first (dn[1 - b], zeroed) adds nothing
            self.tok_zlag.copy_(self.tok_z)
            self._pend_abs = False
            self._lag_base = self.sweeps_done
        _ = VK

    # ---------------------------------------------------------------------------------------------
    def _one_sweep(self) -> None:
        c = self.c
        mode = self._sweep_mode(self.sweeps_done + 1)
        if mode == self.mode and mode in (2, 4) and not self._aux_synced:
            self._sync_aux_z()  # entering a delta mode: z_prev / z_w := z (eager, outside graphs)
        self._aux_synced = self._keeps_aux(mode)
        if mode == 3 and not self._capturing:
            self._ensure_zw()
        # long (chunked) documents add their Δn_dk into ndk[1-a] rows that hold a copy of ndk[a]:
        # every apply -- the previous sweep's, or _prime()'s after init / resume -- seeds that copy
        st = self._state(False)
        inplace = self._inplace_ok and mode in (1, 2, 4)
        if not inplace and self._last_inplace and not self._capturing:
            self._clean_heads()
        if inplace:
            st["dnwk"] = self.nwk  # MODE 1: the sampler's Δ atomics land in n_wk itself
        if self.mh:
            self.mh_build_tables()
            st.update(self.mh_state())
        pending = self._x01_start(self.dn[1 - self.b]) if self._lag_live else None
        if self._guard is not None:
            g = self._guard
            ops.exact_guard(self.ndk[self.a], g["rows"], self.K, g["limit"], g["flag"])
            st["exact_guard"] = g["flag"]
        ops.gibbs_pass(st, self.G, self.KP, self.K, self.alpha, self.cfg.seed, False,
                       self.sweep_ctr, c.chunk_len, host_sweep=self.sweeps_done + 1, mode=mode, sampler=self.qpf,
                       chg_mask=self.wbits if mode == 4 else getattr(self, "chg_mask", None), wpos=c.wpos,
                       z_w=getattr(self, "z_w", None), zz_w=getattr(self, "zz_w", None), alpha_in_row=self._air,
                       mh_doc_moves=getattr(self, "mh_doc_moves", 1), pos_aligned=self._pos_aligned)
        head = self.nwk if inplace else self.dn[self.b][: self.V * self.KS].view(self.V, self.KS)
        if mode == 4:
            # dn[b] head := Δn_wk of the tokens marked in the word-sorted change bitmap
            ops.wdelta_recount(self.wbits, c.wsorted, self.zz_w, head, self.KS)
        elif mode == 0:
            # dn[b] head := this rank's n_wk rebuilt from z (tail keeps Δn_k)
            ops.recount(c.wsorted, c.wslot, self.tok_z, head, self.KS)
        elif mode == 3:
            # dn[b] head := this rank's n_wk, streamed from the word-sorted topic copy
            ops.recount(c.wsorted, None, self.z_w, head, self.KS)
        elif mode == 2:
            # dn[b] head := Δn_wk of the tokens that changed topic this sweep
            ops.delta_recount(c.wslot, c.tile_wlo, c.tile_whi, self.chg_mask, c.tok_word, self.tok_z, self.tok_zprev,
                              head, self.KS, self.G)
        if self._split is not None:
            self._split_delta(self.dn[self.b], self.ndk[self.a], self.ndk[1 - self.a])
        if self._lag_live:
            if self._split is not None:
                # split documents' Δn_dk rows stay synchronous (their rows are doc side)
                self.comm.allreduce_(self.dn[self.b][self._split_off:])
        elif self.comm is not None and self.comm.dist:
            self._allreduce_dn(self.dn[self.b])
        if self._split is not None:
            self._split_apply(self.dn[self.b], self.ndk[self.a], self.ndk[1 - self.a])
        so = self._split_off
        # inside a contiguous averaging window the sample sums gain this sweep's counts in the
        # same launch (int64: no extra pass over n_wk, no separate adds)
        acc = ((self._avg["wk"], self._avg["k"], self._avg["dk"], self.ndk[1 - self.a]) if self._acc else None)
        if self._lag_live:
            # join the collective; add the previous sweep's reduced Δ (absolute if that sweep
            # recounted) and zero its buffer, which the next sweep writes
            self._x01_finish(pending)
            ops.gibbs_apply(self.nwk, self.x01_red[:so], self.dn[1 - self.b][:so], self.nk[self.cn],
                            self.nk[1 - self.cn], self.q, self.qfix, self.V, self.K, self.KS, self.beta, self.vbeta,
                            self.sweep_ctr, bump=True, absolute=self._pend_abs,
                            rows_copy=(self.ndk[1 - self.a], self.ndk[self.a], c.long_rows), acc=acc)
            self._pend_abs = mode in (0, 3)
        else:
            ops.gibbs_apply(self.nwk, self.dn[self.b][:so], self.dn[1 - self.b][:so], self.nk[self.cn],
                            self.nk[1 - self.cn], self.q, self.qfix, self.V, self.K, self.KS, self.beta, self.vbeta,
                            self.sweep_ctr, bump=True, absolute=mode in (0, 3),
                            rows_copy=(self.ndk[1 - self.a], self.ndk[self.a], c.long_rows), acc=acc, inplace=inplace)
        self.a, self.b, self.cn = 1 - self.a, 1 - self.b, 1 - self.cn
        self.sweeps_done += 1
        self._tail_cache = None
        if not self._capturing:
            self._zw_synced = mode == 3
            self._last_inplace = inplace

    def _clean_heads(self) -> None:
        """Zero both Δ heads before a sweep that writes one after in-place sweeps: an in-place apply
        neither reads nor zeroes them, so the head a non-in-place sweep left behind is still there
        (auto mode only switches recount → delta, but a forced or resumed schedule need not)."""
        VK = self.V * self.KS
        for d in self.dn:
            d[:VK].zero_()
        self._last_inplace = False

    def _pair_inplace(self, mode: int) -> bool:
        return self._inplace_ok and mode in (1, 2, 4)

    def _lag_due(self, sweep: int, mode: int) -> bool:
        """Does (1-based) sweep ``sweep`` (of count mode ``mode``) run with the lagged X01?"""
        return self.lag and sweep >= self._lag_from

    def _lag_enter(self) -> None:
        """Start lagging (eager, between sweeps): the counts are current, so the first lagged
        sweep's word side counts every token at tok_z and the Δ it reduces (the buffer the last
        synchronous sweep consumed) must add nothing."""
        self.dn[1 - self.b].zero_()
        self.tok_zlag.copy_(self.tok_z)
        self._pend_abs = False
        self._lag_base = self.sweeps_done
        self._lag_live = True

    def _x01_start(self, src: torch.Tensor):
        """Lagged X01, issued at a sweep's start: x01_red := Σ over ranks of ``src`` (the previous
        sweep's Δ buffer, untouched by this sweep before its apply). The pack (or a copy: the apply
        cannot read and zero one buffer) runs on the compute stream; the collective is issued
        asynchronously, so RCCL runs it on its own stream while this sweep's sampler runs, and
        :meth:`_x01_finish` joins it before the apply -- inside the captured sweep graph too."""
        so = self._split_off
        x = self._x01
        if x is not None:
            ops.x01_pack(src, x["tiny"], x["light"], x["heavy"], self.KS, x["tail_off"], x["tail_len"], x["O8"],
                         x["O"], x["buf"])
            buf = x["buf"]
        else:
            self.x01_red[:so].copy_(src[:so])
            buf = self.x01_red[:so]
        # (no timing events: issue → join spans the sampler; allreduce_ms_per_sweep probes the
        # payload's collective on its own instead)
        h = self.comm.allreduce_async_(buf) if self.comm is not None else None
        if self.comm is not None and self.comm.dist:
            self.timings["allreduce_calls"] += 1
        return h

    def _x01_finish(self, h) -> None:
        if h is not None:
            h.wait()
        x = self._x01
        if x is not None:
            ops.x01_unpack(x["buf"], x["tiny"], x["light"], x["heavy"], self.KS, x["tail_off"], x["tail_len"],
                           x["WO8"], x["WO"], self.x01_red)

    def _lag_drain(self) -> None:
        """End of a sweep() call with the lagged X01: reduce and add the last sweep's Δ (no sample
        is drawn and the sweep counter stays), so n_wk, n_k and q are current again; the next
        sweep's word side then counts every token at tok_z."""
        pb = 1 - self.b
        so = self._split_off
        self._x01_finish(self._x01_start(self.dn[pb]))
        ops.gibbs_apply(self.nwk, self.x01_red[:so], self.dn[pb][:so], self.nk[self.cn], self.nk[1 - self.cn], self.q,
                        self.qfix, self.V, self.K, self.KS, self.beta, self.vbeta, self.sweep_ctr, bump=False,
                        absolute=self._pend_abs)
        # n_k back into the current slot: the sweep parities (a, b, cn) keep their relation, so the
        # captured sweep pairs replay after the drain
        self.nk[self.cn].copy_(self.nk[1 - self.cn])
        self.tok_zlag.copy_(self.tok_z)
        self._pend_abs = False
        self._lag_base = self.sweeps_done  # the next sweep reduces the zeroed buffer: no count
        self._tail_cache = None
        self._avg_cache = None

    def _allreduce_dn(self, buf: torch.Tensor) -> None:
        """X01: all-reduce of the sweep's Δ buffer (Δn_wk ‖ Δn_k replicas ‖ aux words).

        Eager calls are bracketed by HIP events on the compute stream (the RCCL kernel runs on
        the process group's stream, which the compute stream waits on), so the recorded time is
        the device-side time the sweep spends in the collective. Graph-captured sweeps cannot
        carry timing events; :meth:`allreduce_ms_per_sweep` then probes the same payload."""
        timed = (self.device.type == "cuda" and not self._capturing and len(self._ar_events) < 64)
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        x = self._x01
        # a forced 1-rank group (ONI_FORCE_DIST=1: every data-parallel code path on one GPU) keeps
        # the pack / unpack but drops the collective itself -- the sum over one rank is the identity
        # -- unless ONI_COMM_REAL=1 (comm.live), which runs the RCCL all-reduce inside the graph
        reduce = self.comm.live
        if x is not None:
            ops.x01_pack(buf, x["tiny"], x["light"], x["heavy"], self.KS, x["tail_off"], x["tail_len"], x["O8"], x["O"],
                         x["buf"])
            if reduce:
                self.comm.allreduce_(x["buf"])
            ops.x01_unpack(x["buf"], x["tiny"], x["light"], x["heavy"], self.KS, x["tail_off"], x["tail_len"], x["WO8"],
                           x["WO"], buf)
        elif reduce:
            self.comm.allreduce_(buf)
        if timed:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._ar_events.append((e0, e1))
        self.timings["allreduce_calls"] += 1

    def allreduce_bytes_per_sweep(self) -> int:
        """Bytes each rank contributes to X01 per sweep (0 without a process group)."""
        if self.comm is None or not self.comm.dist:
            return 0
        b = self._x01["buf"] if self._x01 is not None else self.dn[0]
        return int(b.numel() * b.element_size())

    def allreduce_ms_per_sweep(self, probe_reps: int = 20) -> float | None:
        """Median device time of the per-sweep Δ all-reduce (ms). Uses the events of eager sweeps;
        when every sweep ran inside a HIP graph, probes ``probe_reps`` all-reduces of a scratch
        buffer of the same size. None without a process group or off-GPU."""
        if self.comm is None or not self.comm.dist or self.device.type != "cuda":
            return None
        times = []
        if self._ar_events:
            self._ar_events[-1][1].synchronize()
            times = [a.elapsed_time(b) for a, b in self._ar_events]
        if not times:
            scratch = torch.zeros_like(self._x01["buf"] if self._x01 is not None else self.dn[0])
            for _ in range(probe_reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                self.comm.allreduce_(scratch)
                e1.record()
                times.append((e0, e1))
            times[-1][1].synchronize()
            times = [a.elapsed_time(b) for a, b in times]
        return round(float(np.median(times)), 4)

    def _graphable(self) -> bool:
        if getattr(self, "_graph_off", False):
            return False  # a capture failed on some rank: eager sweeps for the rest of the model
        if not (self.cfg.use_graph and self.device.type == "cuda" and os.environ.get("ONI_NO_GRAPH", "0") != "1"):
            return False
        if self.comm is None or not self.comm.dist:
            return True
        # RCCL collectives are captured into the sweep graph (the communicator exists: initialize()
        # already all-reduced n_wk); gloo routes through host copies and cannot be captured.
        # Lagged sweeps with live collectives run eagerly: capturing the deferred join of an async
        # RCCL collective crashed in capture_end (hipGraph, ROCm 7.0 RCCL 2.26; tools/lag_real_probe.py)
        if self._lag_live and self.comm.live:
            return False
        return self.comm.graph_capturable() and os.environ.get("ONI_DIST_GRAPH", "1") != "0"

    def _capture(self, mode: int):
        """Capture two sweeps of count mode ``mode`` (parities return to their start) into one HIP graph."""
        saved = (self.a, self.b, self.cn, self.sweeps_done, self._aux_synced, self._pend_abs)
        self._force_mode = mode
        if mode == self.mode:
            self._aux_synced = True  # the eager aux sync happens before the first replay
        s = _capture_stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = torch.cuda.CUDAGraph()
        # capture does not execute: the host-side parities are rewound afterwards (failed or not)
        calls = self.timings["allreduce_calls"]
        self._capturing = True
        # no garbage collection during the capture: a collected CUDAGraph (another model's) would
        # be destroyed mid-capture, which HIP refuses (hipErrorStreamCaptureUnsupported)
        gc_on = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.stream(s):
                # capture_begin/end directly: the torch.cuda.graph() context would synchronize the
                # device and empty the caching allocator first (~1.5 ms per capture, and the day's
                # later allocations then go back to hipMalloc)
                g.capture_begin()
                try:
                    if fault.capture_fails(self.comm.rank if self.comm is not None else 0):
                        raise fault.InjectedFault("injected sweep-graph capture failure")
                    self._one_sweep()
                    self._one_sweep()
                finally:
                    g.capture_end()
        finally:
            self._capturing = False
            self.timings["allreduce_calls"] = calls
            if gc_on:
                gc.enable()
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.a, self.b, self.cn, self.sweeps_done, self._aux_synced, self._pend_abs = saved
            self._force_mode = None
        entry = (g, (self.a, self.b, self.cn))
        self._graphs[(mode, self._acc, self._lag_live)] = entry
        return entry

    def _capture_agreed(self, mode: int, also: int | None = None):
        """Capture the ``mode`` pair (and the ``also`` pair), then vote: the graphs are used only if
        every rank captured (comm.Comm.agree, an eager MIN all-reduce -- captures happen at the same
        sweep on every rank, so the votes line up). Otherwise every rank drops its graphs and runs
        eager sweeps from here on: the same kernels and collectives in the same order, so the chain
        is unchanged. Returns the ``mode`` entry, or None after a fallback."""
        err = None
        entry = None
        try:
            entry = self._capture(mode)
            if also is not None:
                self._capture(also)
        except Exception as e:  # noqa: BLE001 -- any capture error (HIP, RCCL, injected) falls back
            err = e
        ok = err is None
        if self.comm is not None and self.comm.dist:
            ok = self.comm.agree(ok)
        if ok:
            return entry
        import sys
        why = repr(err) if err is not None else "another rank's capture failed"
        sys.stderr.write(f"[oni355] sweep-graph capture failed ({why}): eager sweeps from sweep "
                         f"{self.sweeps_done + 1}\n")
        self.timings["graph_fallback"] = why
        self._graphs = {}
        self._graph = None
        self._graph_off = True
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return None

    @traced("oni:lda.sweeps")
    def sweep(self, n: int = 1) -> None:
        """Run ``n`` sweeps (graph-replayed in same-mode pairs on a single GPU)."""
        fault.maybe_inject(self.sweeps_done, self.comm.rank if self.comm else 0, corrupt=self._corrupt)
        if self._graph is None:
            self._graphs = {}
        if self._watchdog is not None:
            self._watchdog.arm()
        try:
            while n > 0:
                nxt = [p for p in self._avg_at if p > self.sweeps_done]
                contiguous = self._avg is not None and int(self.cfg.post_every) == 1
                if nxt and contiguous and self.sweeps_done + 1 >= nxt[0]:
                    # inside a contiguous window: every sweep adds its sample, in the graph
                    self._ensure_avg()
                    seg = min(n, self._avg_at[-1] - self.sweeps_done)
                    self._acc = True
                    try:
                        self._sweep_n(seg)
                    finally:
                        self._acc = False
                    self._avg["n"] += seg
                    self._avg_cache = None
                    n -= seg
                    continue
                if nxt and contiguous:
                    seg = min(n, nxt[0] - 1 - self.sweeps_done)
                else:
                    seg = min(n, nxt[0] - self.sweeps_done) if nxt else n
                self._sweep_n(seg)
                n -= seg
                if not contiguous and self._avg is not None and self.sweeps_done in self._avg_at:
                    self._add_sample()
            if self._lag_live:
                self._lag_drain()
        finally:
            if self._watchdog is not None:
                self._watchdog.disarm()
        if self.cfg.check_invariants:
            self.check_invariants()
        if self.cfg.health_check:
            self.check_health()

    def _corrupt(self) -> None:
        """ONI_FAULT kind:nan -- poison the state the way a bad DMA / bit flip would: a negative
        doc-topic count (carried from sweep to sweep by the sampler) and a NaN in the q table."""
        if self.c.D:
            self.ndk_cur[0, 0] = -1 - self.ndk_cur[0, 0].abs()
        self.q[0, 0] = float("nan")
        self._corrupted = True
        self._tail_cache = None

    def check_health(self) -> None:
        """Numerical health check after every ``sweep()`` call (one device reduction, one host
        read): finite q table, no negative word-topic / topic / doc-topic count. Raises
        fault.NumericalFault (the supervisor then restarts from the last good checkpoint)."""
        K = self.K
        if self.device.type == "cuda":
            t = self._tail()[1]
            extra = False
            if self.c.D > self.c.D_own:  # split-document pieces: rows past D_own
                extra = bool((self.ndk_cur[self.c.D_own: self.c.D, :K] < 0).any())
            flags = [t[4] > 0, t[5] > 0, t[6] > 0 or extra]
            if any(flags):
                raise fault.NumericalFault(f"corrupt model state after sweep {self.sweeps_done}: non-finite "
                                           f"q={flags[0]}, negative counts={flags[1] or flags[2]}")
            return
        flags = torch.stack([
            (~torch.isfinite(self.q[:, :K])).any(),
            (self.nk_cur[:K] < 0).any() | (self.nwk[:, :K] < 0).any(),
            (self.ndk_cur[: self.c.D, :K] < 0).any() if self.c.D else torch.zeros((), dtype=torch.bool,
                                                                                   device=self.device),
        ]).cpu().tolist()
        if any(flags):
            raise fault.NumericalFault(f"corrupt model state after sweep {self.sweeps_done}: non-finite q={flags[0]}, "
                                       f"negative counts={flags[1] or flags[2]}")

    def close(self) -> None:
        """Stop the watchdog thread and release the captured sweep graphs (training finished): a
        graph destroyed later, by the cyclic garbage collector, could land inside the next model's
        capture, where HIP refuses the destruction. A later sweep() recaptures."""
        if self._watchdog is not None:
            self._watchdog.close()
            self._watchdog = None
        self._graph = None
        self._graphs = {}

    def check_invariants(self) -> None:
        """Debug-mode count invariants: Σn_wk = Σn_k = global tokens, Σn_dk = local
        tokens, no negative count, n_k = column sums of n_wk. Raises AssertionError."""
        K = self.K
        T_loc = torch.tensor([float(self.c.T)], dtype=torch.float64, device=self.device)
        # rows [0, D_own) are this rank's documents (split documents held whole by their primary)
        T_rows = int(self.c.split["own_tokens"]) if self.c.split is not None else int(self.c.T)
        T_glob = T_loc.clone()
        if self.comm is not None and self.comm.dist:
            self.comm.allreduce_(T_glob)
        nwk = self.nwk[:, :K].to(torch.int64)
        nk = self.nk_cur[:K].to(torch.int64)
        ndk = self.ndk_cur[: self.c.D_own, :K].to(torch.int64)
        tg, tl = int(T_glob.item()), T_rows
        assert int(nwk.min()) >= 0 and int(ndk.min()) >= 0 and int(nk.min()) >= 0, "negative count"
        assert int(nwk.sum()) == tg, f"sum n_wk {int(nwk.sum())} != tokens {tg}"
        assert torch.equal(nwk.sum(0), nk), "n_k != column sums of n_wk"
        assert int(nk.sum()) == self.T_global, "Σ n_k != token count"
        assert int(ndk.sum()) == tl, f"sum n_dk {int(ndk.sum())} != local tokens {tl}"
        assert not bool(self.nwk[:, K:].any()) and not bool(self.ndk_cur[:, K:].any()), "padding topics used"

    def _sweep_n(self, n: int) -> None:
        done = 0
        while done < n:
            self._decide_mode()
            m1 = self._sweep_mode(self.sweeps_done + 1)
            m2 = self._sweep_mode(self.sweeps_done + 2)
            if not self._lag_live and self._lag_due(self.sweeps_done + 1, m1):
                self._lag_enter()
            # a lagged pair's first apply adds the previous sweep's Δ: same absoluteness as m1's
            # (and a pair never straddles the start of the lag)
            lag_off = self.lag and (self._lag_due(self.sweeps_done + 1, m1) != self._lag_due(self.sweeps_done + 2, m2)
                                    or (self._lag_live and self._pend_abs != (m1 in (0, 3))))
            if not (self._graphable() and n - done >= 2 and m1 == m2) or lag_off:
                self._one_sweep()
                self._note_changes()
                done += 1
                continue
            if m1 == self.mode and m1 in (2, 4) and not self._aux_synced:
                self._sync_aux_z()
            if m1 == 3:
                self._ensure_zw()
            entry = self._graphs.get((m1, self._acc, self._lag_live))
            if entry is not None and entry[1] != (self.a, self.b, self.cn):
                self._one_sweep()  # realign parities with the captured pair
                self._note_changes()
                done += 1
                continue
            if entry is None and not self._graphs and not self._eager_lead_done and n - done >= 4 \
                    and os.environ.get("ONI_GRAPH_EAGER_LEAD", "1") == "1":
                # the first capture of a model costs ~0.26 ms of host time with nothing queued: run
                # this pair eagerly first, so that the device works through it while the host
                # captures (eager and replayed sweeps draw the same chain)
                self._eager_lead_done = True
                for _ in range(2):
                    self._one_sweep()
                    self._note_changes()
                done += 2
                continue
            if entry is None:
                # capture the delta pair now too: no capture stall at the switch
                also = (self.mode if (self.auto and self.cfg.auto_switch == 0 and m1 == self.early and not self.lag
                                      and (self.mode, self._acc, False) not in self._graphs) else None)
                entry = self._capture_agreed(m1, also)
                if entry is None:
                    continue  # fell back to eager sweeps (every rank)
            if not self._pair_inplace(m1) and self._last_inplace:
                self._clean_heads()  # eager, before the replay (see _clean_heads)
            self._graph = entry[0]
            entry[0].replay()
            self._last_inplace = self._pair_inplace(m1)
            if self._lag_live:
                self._pend_abs = m1 in (0, 3)
            self.timings["graph_replays"] = self.timings.get("graph_replays", 0) + 1
            self.sweeps_done += 2
            self._aux_synced = self._keeps_aux(m1)
            self._zw_synced = m1 == 3
            self._note_changes()
            done += 2
            if self._watchdog is not None:
                self._watchdog.kick()

    # ---- posterior averaging -------------------------------------------------------------------
    def plan_average(self, total_sweeps: int) -> None:
        """Average the counts of the samples at sweeps total, total - e, …, total - (S-1)·e
        (e = cfg.post_every, S = cfg.post_samples capped at total / 4e)."""
        S, e = max(1, int(self.cfg.post_samples)), max(1, int(self.cfg.post_every))
        # at most the last quarter of the chain (burn-in first): a 200-sweep day averages the 50
        # samples of sweeps 151-200, a 30-sweep run 7, a run of < 8 sweeps none. ONI_POST_SPAN
        # (default 0.25) sets that fraction.
        span = float(os.environ.get("ONI_POST_SPAN", "0.25"))
        S = min(S, int(int(total_sweeps) * span) // e)
        at = [total_sweeps - j * e for j in range(S) if total_sweeps - j * e > 0]
        self._avg_at = sorted(at) if S > 1 else []
        self._avg_cache = None
        dev = self.device
        # the sums are allocated at the first sample (_ensure_avg), when the counts they bound exist
        self._avg = dict(n=0, wk=None, k=None, dk=None) if self._avg_at else None
        _ = dev

    def _ensure_avg(self) -> None:
        """Allocate the sample sums. S samples of an int32 count wrap an int32 sum once the count
        passes 2^31 / S (43M at S = 50: one topic's share of a config-4/5 corpus), so each table is
        int64 when S times its largest possible entry could pass 2^31 -- n_k: the global token
        count; n_wk: the largest global word count; n_dk: the longest document row -- and int32
        otherwise (the default day: half the bytes in k_apply's fused add). ONI_POST_WIDE=1 forces
        int64."""
        a = self._avg
        if a is None or a["wk"] is not None:
            return
        S, K, dev = len(self._avg_at), self.K, self.device
        force = os.environ.get("ONI_POST_WIDE", "0") == "1"
        wk_max = int(self.nwk[:, :K].sum(1, dtype=torch.int64).max()) if self.nwk.shape[0] else 0
        dk_max = int(self.ndk_cur[:, :K].sum(1, dtype=torch.int64).max()) if self.c.D else 0

        def dt(bound: int):
            return torch.int64 if force or bound * S > INT32_COUNT_MAX else torch.int32
        a["wk"] = torch.zeros(self.nwk.shape, dtype=dt(wk_max), device=dev)
        a["k"] = torch.zeros(self.nk[0].shape, dtype=dt(max(self.T_global, int(self.nk_cur[:K].max()))), device=dev)
        a["dk"] = torch.zeros(self.ndk[0].shape, dtype=dt(dk_max), device=dev)

    @property
    def average_window(self) -> tuple[int, int] | None:
        """(first, last) sample sweep of the planned average, or None."""
        return (self._avg_at[0], self._avg_at[-1]) if self._avg_at else None

    def average_state(self) -> dict | None:
        """The accumulated samples (for a checkpoint; the K real topics only, so the state does
        not depend on the kernel tiling's padding), or None outside an averaging window."""
        a = self._avg
        if a is None or a["n"] == 0:
            return None
        K = self.K
        return {"n": int(a["n"]), "wk": a["wk"][:, :K].cpu().to(torch.int64), "k": a["k"][:K].cpu().to(torch.int64),
                "dk": a["dk"][:, :K].cpu().to(torch.int64)}

    def load_average_state(self, st: dict) -> None:
        """Restore :meth:`average_state` (same documents and vocabulary) after a resume inside the
        window."""
        a = self._avg
        if a is None:
            raise ValueError("checkpoint holds posterior-averaging samples but no average is planned")
        self._ensure_avg()
        K = self.K
        for k in ("wk", "k", "dk"):
            want = (a[k].shape[0], K) if a[k].dim() == 2 else (K,)
            v = st[k]
            # states saved before the K-column format hold the KS-wide tiling-padded tables (the
            # padding topics are never used): their first K columns are the same sums
            if tuple(v.shape[:-1]) == want[:-1] and v.shape[-1] == self.KS and self.KS != K:
                v = v[..., :K]
            if tuple(v.shape) != want:
                raise ValueError(f"averaging state {k} shape {tuple(st[k].shape)} != {want}")
            a[k].zero_()
            a[k][..., :K].copy_(v.to(a[k].device))
        a["n"] = int(st["n"])
        self._avg_cache = None

    def _accumulate(self) -> None:
        """Add the current counts to the (int64) sample sums: samples taken every post_every > 1
        sweeps, outside the graphs (contiguous windows add inside k_apply)."""
        self._ensure_avg()
        a = self._avg
        a["wk"] += self.nwk
        a["k"] += self.nk_cur
        a["dk"] += self.ndk_cur

    def _add_sample(self) -> None:
        self._accumulate()
        self._avg["n"] += 1
        self._avg_cache = None

    def _averaged(self):
        """(θ, φ) from the accumulated samples, once every planned sample is in; else None."""
        a = self._avg
        if a is None or a["n"] == 0 or a["n"] != len(self._avg_at) or self.sweeps_done != self._avg_at[-1]:
            return None
        if self._avg_cache is None and self.device.type == "cuda":
            S, K = float(a["n"]), self.K
            th = ops.theta_rows(a["dk"], K, S * self.alpha, S * K * self.alpha)
            ph = ops.phi_rows(a["wk"], a["k"], K, S * self.beta, float(np.float32(S) * np.float32(self.vbeta)))
            self._avg_cache = (th, ph)
        if self._avg_cache is None:
            S, K = float(a["n"]), self.K
            n = a["dk"].to(torch.float32)
            nd = a["dk"][:, :K].to(torch.int64).sum(1, keepdim=True).to(torch.float32)  # as k_theta_rows
            th = (n + S * self.alpha) / (nd + S * K * self.alpha)
            th[:, K:] = 0
            den = a["k"].to(torch.float32) + np.float32(S) * self.vbeta
            ph = (a["wk"].to(torch.float32) + S * self.beta) / den
            ph[:, K:] = 0
            self._avg_cache = (th.contiguous(), ph.contiguous())
        return self._avg_cache

    # ---------------------------------------------------------------------------------------------
    @property
    def ndk_cur(self) -> torch.Tensor:
        return self.ndk[self.a]

    @property
    def nk_cur(self) -> torch.Tensor:
        return self.nk[self.cn]

    def theta(self) -> torch.Tensor:
        """θ[d,k] = (n_dk+α)/(n_d+Kα), padded to KS with zeros (score-kernel layout); from the
        averaged counts once the planned posterior average is complete (:meth:`plan_average`)."""
        avg = self._averaged()
        if avg is not None:
            return avg[0]
        if self.device.type == "cuda":
            return ops.theta_rows(self.ndk_cur, self.K, self.alpha, self.K * self.alpha)
        n = self.ndk_cur.to(torch.float32)
        nd = self.ndk_cur[:, : self.K].to(torch.int64).sum(1, keepdim=True).to(torch.float32)
        th = (n + self.alpha) / (nd + self.K * self.alpha)
        th[:, self.K:] = 0
        return th.contiguous()

    def phi(self) -> torch.Tensor:
        """φ[w,k] = (n_wk+β)/(n_k+Vβ) for the current counts (= the q table), KS-padded; from the
        averaged counts once the planned posterior average is complete."""
        avg = self._averaged()
        return avg[1] if avg is not None else self.q

    @traced("oni:lda.loglik")
    def log_likelihood(self) -> float:
        """Collapsed joint log p(w, z) (Griffiths & Steyvers 2004), summed over ranks."""
        K, a, b, V = self.K, self.alpha, self.beta, self.V
        if self.device.type == "cuda":
            dev_t, host = self._tail()
            cw = K * (math.lgamma(V * b) - V * math.lgamma(b))
            cd = self.c.D_own * (math.lgamma(K * a) - K * math.lgamma(a))
            if self.comm is not None and self.comm.dist:
                doc_v = (dev_t[2] - dev_t[3] + cd).reshape(1)
                self.comm.allreduce_(doc_v)
                return float(cw + host[0] - host[1] + float(doc_v.cpu()[0]))
            return float(cw + host[0] - host[1] + (cd + host[2] - host[3]))
        nwk = self.nwk[:, :K].to(torch.float64)
        nk = self.nk_cur[:K].to(torch.float64)
        word = (K * (math.lgamma(V * b) - V * math.lgamma(b)) + torch.lgamma(nwk + b).sum()
                - torch.lgamma(nk + V * b).sum())
        D_own = self.c.D_own
        ndk = self.ndk_cur[:D_own, :K].to(torch.float64)
        nd = ndk.sum(1)
        doc = (D_own * (math.lgamma(K * a) - K * math.lgamma(a)) + torch.lgamma(ndk + a).sum()
               - torch.lgamma(nd + K * a).sum())
        doc_v = doc.reshape(1)
        if self.comm is not None and self.comm.dist:
            self.comm.allreduce_(doc_v)
        return float(word + doc_v[0])

    def _tail(self):
        """(device [8] tail sums, host list) of the current counts: log-likelihood lgamma sums and
        health counts in one fused pass (ops.tail_sums), computed once per model state -- the
        health check at the end of sweep() and the likelihood after training share it."""
        if self._tail_cache is None or self._tail_cache[0] != self.sweeps_done:
            t = ops.tail_sums(self.nwk, self.q, self.nk_cur, self.ndk_cur, self.c.D_own, self.K, self.alpha,
                              self.beta, self.vbeta)
            self._tail_cache = (self.sweeps_done, t, t.cpu().tolist())
        return self._tail_cache[1], self._tail_cache[2]

    def record_likelihood(self) -> float:
        ll = self.log_likelihood()
        if not math.isfinite(ll):
            raise fault.NumericalFault(f"non-finite log-likelihood {ll} after sweep {self.sweeps_done}")
        self.likelihoods.append((self.sweeps_done, ll))
        return ll

    # ---------------------------------------------------------------------------------------------
    def canonical_z(self) -> torch.Tensor:
        c = self.c
        out = torch.zeros(max(c.T, 1), dtype=torch.uint8, device=self.device)
        ops.sell_perm_z(c.chunk_doc, c.chunk_pos0, c.chunk_len, c.S, c.slice_off, c.doc_tok_ptr, self.tok_z, out,
                        True)
        return out[: c.T]

    def load_canonical_z(self, z: torch.Tensor, sweeps_done: int, counts_from: "GibbsLDA | None" = None) -> None:
        """Resume: scatter z into SELL, recount every table from z, refresh q (bitwise resume).

        ``counts_from``: a model of another tiling over the same documents and tokens whose chain
        ``z`` is (the MH model's dense burn-in, pipeline.common.build_and_train): its count tables
        -- current at the end of every sweep -- are copied instead of recounted (125M index adds
        and two all-reduces less)."""
        c = self.c
        zc = torch.zeros(max(c.T, 1), dtype=torch.uint8, device=self.device)
        zc[: c.T] = z.to(self.device)
        self.tok_z.zero_()
        ops.sell_perm_z(c.chunk_doc, c.chunk_pos0, c.chunk_len, c.S, c.slice_off, c.doc_tok_ptr, self.tok_z, zc,
                        False)
        for t in (*self.ndk, self.nwk, *self.nk, *self.dn):
            t.zero_()
        K, KS = self.K, self.KS
        o = counts_from
        if o is not None and o.K == K and o.nwk.shape[0] == self.nwk.shape[0] and o.ndk_cur.shape[0] == self.ndk[0].shape[0]:
            self.ndk[0][:, :K].copy_(o.ndk_cur[:, :K])
            self.nwk[:, :K].copy_(o.nwk[:, :K])
            self.nk[0][:K].copy_(o.nk_cur[:K])
        else:
            tdoc, tword = canonical_tokens(c)
            zz = zc[: c.T].to(torch.int64)
            self.ndk[0].view(-1).index_add_(0, tdoc * KS + zz, torch.ones_like(zz, dtype=torch.int32))
            self.nwk.view(-1).index_add_(0, tword * KS + zz, torch.ones_like(zz, dtype=torch.int32))
            self.nk[0].index_add_(0, zz, torch.ones_like(zz, dtype=torch.int32))
            self._split_sync_absolute(self.ndk[0])
            if self.comm is not None and self.comm.dist:
                self.comm.allreduce_(self.nwk)
                self.comm.allreduce_(self.nk[0])
        self._sync_aux_z()
        self.a = self.b = self.cn = 0
        self.sweeps_done = sweeps_done
        self.T_global = int(self.nk[0][: self.K].sum())
        self._check_magnitude()
        self._delta_on = False
        self._chg_q = []
        self._poll_off = False
        self._graph = None
        self._prime()
