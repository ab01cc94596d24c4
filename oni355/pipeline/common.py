"""Source-independent stages of suspicious-connects: vocabulary, owner routing, corpus, LDA,
scoring and top-N selection (the oni-ml pre-LDA / LDA / post-LDA skeleton).

Data-parallel layout: every rank featurizes its own events; tokens are
routed to the rank that owns their document (hash of the document key), so each rank's corpus is
document-complete and the sampler needs only the per-sweep Δn_wk all-reduce. Word ids come from
one global sorted vocabulary (all-gather of local unique keys, X02), so ids -- and therefore every
sample -- are independent of the GPU count.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..utils.obs import StageTimer, traced
from ..models.corpus import Corpus, auto_chunk_len, build_corpus
from ..models.gibbs import GibbsConfig, GibbsLDA
from ..parallel.comm import Comm

U32MASK = 0xFFFFFFFF


def u32_to_i64(t: torch.Tensor) -> torch.Tensor:
    """int32 tensor holding u32 bits → non-negative int64."""
    return t.to(torch.int64) & U32MASK


def i64_to_u32bits(t: torch.Tensor) -> torch.Tensor:
    return (t & U32MASK).to(torch.int64).to(torch.int32) if t.dtype == torch.int64 else t


@traced("oni:vocab")
def encode_words(word_keys64: torch.Tensor, comm: Comm | None, key_bits: int = 64):
    """(global sorted vocabulary int64, int32 word id of every key) -- K08 + collective X02.

    On a GPU the local dictionary is the native radix-sort encoder (ops.corpus.dict_encode, sorting
    only ``key_bits`` bits); with a process group the local unique keys are all-gathered and merged,
    and local ids are remapped through the (small) local-unique → global table."""
    if word_keys64.is_cuda:
        from ..ops import corpus as oc
        luniq, lids = oc.dict_encode(word_keys64.contiguous(), key_bits, hashed=True)
    else:
        luniq, inv = torch.unique(word_keys64, return_inverse=True)
        lids = inv.to(torch.int32)
    if comm is None or not comm.dist:
        return luniq, lids
    parts = comm.allgather_var(luniq)
    vocab = torch.unique(torch.cat([p.to(luniq.device) for p in parts]))
    remap = torch.searchsorted(vocab, luniq).to(torch.int32)
    return vocab, remap[lids.long()]


def global_vocab(keys64: torch.Tensor, comm: Comm | None) -> torch.Tensor:
    """Sorted unique int64 word keys over all ranks (collective X02)."""
    return encode_words(keys64, comm)[0]


def encode_docs(doc_keys64: torch.Tensor, key_bits: int = 32):
    """(sorted unique doc keys int64, int32 doc id of every token)."""
    if doc_keys64.is_cuda:
        from ..ops import corpus as oc
        return oc.dict_encode(doc_keys64.contiguous(), key_bits)
    u, inv = torch.unique(doc_keys64, return_inverse=True)
    return u, inv.to(torch.int32)


def doc_owner(doc_keys64: torch.Tensor, world: int) -> torch.Tensor:
    """Owner rank of each document: multiplicative hash of the u32 key (spreads /24 subnets)."""
    h = (doc_keys64 * 0x9E3779B1) & U32MASK
    return ((h >> 16) % world).to(torch.int64)


HEAVY_DOCS_PER_RANK = 4096
PLACEMENT_BUCKETS_PER_RANK = 64


def lpt_place(counts: np.ndarray, load: np.ndarray) -> np.ndarray:
    """Longest-processing-time greedy: each count (already in placement order) goes to the rank
    with the smallest load so far, ties to the lowest rank. ``load`` is updated in place.
    Native (csrc/native/placement.cpp); the NumPy loop is the reference used when the host
    library is absent."""
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    owner = np.zeros(counts.size, dtype=np.int32)
    try:
        from ..ops import native
        L = native.lib()
        fn = L.oni_lpt_place
    except (RuntimeError, AttributeError):
        fn = None
    if fn is not None:
        import ctypes as C
        fn.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p]
        fn.restype = C.c_int
        if fn(counts.ctypes.data, counts.size, int(load.size), load.ctypes.data, owner.ctypes.data):
            raise ValueError("oni_lpt_place: bad arguments")
        return owner
    for i, c in enumerate(counts.tolist()):
        r = int(np.argmin(load))
        load[r] += c
        owner[i] = r
    return owner


def place_docs(doc_keys64: torch.Tensor, weights: torch.Tensor | None, comm: Comm, per_doc: bool = False):
    """Owner rank of each token's document, balanced by global token counts.

    IP documents are power-law sized (one synthetic 100M-flow day puts ~8 % of all tokens on a
    single IP), so a plain hash leaves the busiest rank ~1.5× the mean at 8 ranks and every sweep
    waits for it. Every rank proposes its ``HEAVY_DOCS_PER_RANK`` locally heaviest documents; the
    union of the proposals gets exact global counts (one all-reduce over the candidates, not an
    all-gather of every document); every other document falls into one of
    ``PLACEMENT_BUCKETS_PER_RANK × world`` hash buckets, and candidates and buckets together are
    placed by longest-processing-time greedy (:func:`lpt_place`). Collective volume is
    O(candidates · world), independent of the number of documents.
    Deterministic on every rank (same candidate set and counts; order count desc, key asc; ties →
    lowest rank); results stay world-size invariant because the sampler's chain never depends on
    placement. Returns the owner of every token, or with ``per_doc`` (owner of every local
    document int32, document id of every token int32, sorted unique local doc keys int64)."""
    W = comm.world
    dev = doc_keys64.device
    if doc_keys64.is_cuda:
        from ..ops import corpus as oc
        ukeys, inv, ucnt = oc.dict_encode(doc_keys64.contiguous(), 32,
                                          weights.to(torch.int32) if weights is not None else None, counts=True)
    else:
        ukeys, inv = encode_docs(doc_keys64.contiguous())
        w = weights.to(torch.int64) if weights is not None else torch.ones(inv.numel(), dtype=torch.int64)
        ucnt = torch.zeros(ukeys.numel(), dtype=torch.int64).index_add_(0, inv.long(), w)
    U = int(ukeys.numel())
    # local proposals: heaviest first, ties by key (ukeys is ascending, the sort is stable)
    top = torch.argsort(ucnt, descending=True, stable=True)[: min(HEAVY_DOCS_PER_RANK, U)]
    cand = torch.unique(torch.cat([p.to(dev) for p in comm.allgather_var(ukeys[top].contiguous())]))
    if U:
        pos = torch.searchsorted(ukeys, cand).clamp_(max=U - 1)
        hit = ukeys[pos] == cand
    else:
        pos = torch.zeros_like(cand)
        hit = torch.zeros(cand.numel(), dtype=torch.bool, device=dev)
    ccnt = torch.where(hit, ucnt[pos] if U else torch.zeros_like(cand), torch.zeros_like(cand))
    is_cand = torch.zeros(U, dtype=torch.bool, device=dev)
    is_cand[pos[hit]] = True
    # all other documents are hashed into B buckets that are placed like documents, so the rank
    # that takes a huge IP takes correspondingly fewer light ones
    B = PLACEMENT_BUCKETS_PER_RANK * W
    hb = doc_owner(ukeys, B)
    bload = torch.zeros(B, dtype=torch.int64, device=dev).index_add_(0, hb[~is_cand], ucnt[~is_cand])
    both = torch.cat([ccnt, bload])  # one collective for candidate counts + bucket loads
    comm.allreduce_(both)
    nc = int(cand.numel())
    o = torch.argsort(both, descending=True, stable=True)  # candidates (by key) before buckets on ties
    assign = lpt_place(both[o].cpu().numpy(), np.zeros(W, dtype=np.int64))
    iown = torch.empty(nc + B, dtype=torch.int64)
    iown[o.cpu()] = torch.from_numpy(assign.astype(np.int64))
    iown = iown.to(dev)
    uown = iown[nc:][hb]
    uown[pos[hit]] = iown[:nc][hit]
    if per_doc:
        return uown.to(torch.int32), inv, ukeys
    return uown[inv.long()]


def balanced_owner(doc_keys64: torch.Tensor, weights: torch.Tensor, comm: Comm) -> torch.Tensor:
    """Alias of :func:`place_docs` (round-1 name)."""
    return place_docs(doc_keys64, weights, comm)


@dataclass
class Route:
    """How this rank's tokens were sent to their document owners (for the way back)."""
    order: torch.Tensor     # int [n_sent]: slot i of the owner-grouped send buffer holds token order[i]
    send_counts: list       # tokens sent to each rank
    recv_counts: list       # tokens received from each rank (the owner side's layout)


@traced("oni:route_to_owners")
def route_to_owners(doc_keys64: torch.Tensor, word_ids: torch.Tensor, weights: torch.Tensor | None,
                    comm: Comm | None):
    """Send each token to its document's owner rank and dictionary-encode the owner's documents.

    Returns (sorted unique owner-local doc keys int64, doc id int32, word id int32, weight int32
    of every received token, Route) -- what ``encode_docs`` of the received keys would give.

    GPU: the sender already holds its documents' dictionary (:func:`place_docs`), so each owner
    gets the sorted list of the document keys it owns from every source (one small alltoallv,
    ≤ the local distinct documents) and the tokens carry an index into that list (packed int32
    columns: 8 B per token, 12 B with weights). The owner then dictionary-encodes only the
    concatenated key lists (Σ per-source distinct docs, not its ~T/W tokens) and maps every token
    through them in one kernel (``route_unpack``). CPU: the tokens carry their keys."""
    if comm is None or not comm.dist:
        w = weights if weights is not None else torch.ones_like(word_ids, dtype=torch.int32)
        udoc, inv = encode_docs(doc_keys64)
        return udoc, inv, word_ids, w, None
    if doc_keys64.is_cuda:
        from ..ops import corpus as oc
        uown, ids, ukeys = place_docs(doc_keys64, weights, comm, per_doc=True)
        U = int(ukeys.numel())
        # key lists per owner: the local docs grouped by owner, ascending keys inside a group
        kperm = torch.argsort(uown, stable=True)
        kcounts = torch.bincount(uown.long(), minlength=comm.world)
        kstart = _excl_cumsum(kcounts)
        pos = torch.empty(U, dtype=torch.int32, device=ukeys.device)
        pos[kperm] = (torch.arange(U, dtype=torch.int64, device=ukeys.device)
                      - kstart[uown[kperm].long()]).to(torch.int32)
        ksend = i64_to_u32bits(ukeys[kperm]).to(torch.int32).contiguous()
        send, order, counts = oc.route_pack_ids(uown, ids, pos, word_ids.to(torch.int32).contiguous(),
                                                weights, comm.world)
        # both count vectors travel in one small exchange, then the two payload alltoallvs
        sc = torch.stack([counts.to(torch.int64), kcounts.to(torch.int64)], 1).reshape(-1).contiguous()
        rcm = comm.alltoallv(sc.view(comm.world, 2), [1] * comm.world, recv_counts=[1] * comm.world).reshape(-1).tolist()
        rc, krc = rcm[0::2], rcm[1::2]
        scl, kcl = counts.tolist(), kcounts.tolist()
        rkeys = comm.alltoallv(ksend, kcl, recv_counts=krc)
        recv = comm.alltoallv(send, scl, recv_counts=rc)
        udoc, kid = encode_docs(u32_to_i64(rkeys.view(-1)).contiguous())
        inv, wi, wt = oc.route_unpack(recv.contiguous(), rc, krc, kid, weights is not None)
        return udoc, inv, wi, wt, Route(order, scl, rc)
    owner = place_docs(doc_keys64, weights, comm)
    order = torch.argsort(owner, stable=True)
    counts = torch.bincount(owner, minlength=comm.world)
    cols = [i64_to_u32bits(doc_keys64[order]), word_ids[order].to(torch.int32)]
    if weights is not None:
        cols.append(weights[order].to(torch.int32))
    send = torch.stack(cols, 1).contiguous()
    recv, rc = comm.alltoallv(send, counts, return_recv_counts=True)
    dk = u32_to_i64(recv[:, 0])
    wi = recv[:, 1].contiguous()
    wt = recv[:, 2].contiguous() if weights is not None else torch.ones_like(wi)
    udoc, inv = encode_docs(dk)
    return udoc, inv, wi, wt, Route(order, counts.tolist(), rc)


def return_to_origin(x: torch.Tensor, route: Route, comm: Comm) -> torch.Tensor:
    """Inverse of :func:`route_to_owners` for a per-received-token value ``x`` (owner layout):
    returns the value of every token this rank sent, in its original token order."""
    back = comm.alltoallv(x.contiguous(), route.recv_counts, recv_counts=route.send_counts)
    out = torch.empty_like(back)
    out[route.order.to(back.device).long()] = back
    return out


@dataclass
class LdaRun:
    corpus: Corpus
    model: GibbsLDA
    doc_keys64: torch.Tensor  # sorted unique local doc keys (row i of θ)
    vocab: torch.Tensor        # sorted global word keys (row i of φ)
    timings: dict = field(default_factory=dict)
    # the corpus PairSet (ops.corpus.PairSet on a GPU, TorchPairs on the CPU): world 1 on a GPU it
    # is also the events' score plan (K15); with a process group it maps every received token to
    # its (doc, word) pair for owner-side scoring (owner_token_scores)
    pairs: object = None
    route: Route | None = None  # with a process group: how this rank's tokens went to their owners


@traced("oni:build_and_train")
def build_and_train(doc_keys64: torch.Tensor, word_keys64: torch.Tensor | None, weights: torch.Tensor | None,
                    vocab: torch.Tensor, K: int, alpha: float | None, beta: float, seed: int, sweeps: int,
                    chunk_len: int, comm: Comm | None, eval_every: int = 0, burnin: int = 0, ckpt=None, log=None,
                    train: bool = True, timer: StageTimer | None = None, ldac_dir: str | None = None,
                    ldac_lag: int = 0, word_ids: torch.Tensor | None = None, n_event0: int = 0,
                    on_train=None) -> LdaRun:
    """Token keys → owner routing → local corpus → Gibbs LDA trained for ``sweeps`` sweeps.

    ``word_ids`` (int32, from :func:`encode_words`) skips the vocabulary lookup of ``word_keys64``.
    ``n_event0``: the first ``n_event0`` tokens are the events' first endpoints (world 1: the
    corpus pair build then also yields the score plan's event order, see :func:`plan_from_pairs`).
    ``ldac_dir`` + ``ldac_lag`` > 0 emit lda-c ``NNN.{beta,gamma,other}`` snapshots every
    ``ldac_lag`` sweeps (oni-lda-c's LAG); ``final.*`` is written by the caller.
    ``burnin``: sweeps before the chain is considered mixed -- the ``eval_every`` likelihood trace
    and the LAG snapshots only sample sweeps after it (BURNIN in duxbay.conf / ``burnin`` in the
    lda-c settings file); θ/φ always come from the final sweep.
    ``on_train()`` is called as the sweeps start (e.g. to queue the next day's upload on a copy
    stream: training needs no host↔device transfers, while the collectives of the earlier stages
    would wait behind a bulk copy on the DMA engine)."""
    dev = doc_keys64.device
    timer = timer or StageTimer(dev)
    dist_on = comm is not None and comm.dist
    with timer.stage("corpus"):
        if word_ids is None:
            word_ids = torch.searchsorted(vocab, word_keys64).to(torch.int32)
        use_w = weights is not None
        udoc, inv, wi, wt, route = route_to_owners(doc_keys64, word_ids, weights, comm)
        G, _ = ops.choose_tiling(K)
        if chunk_len <= 0:
            T_glob = float(wt.sum()) if wt.numel() else 0.0
            if dist_on:
                T_glob = comm.allreduce_scalar(T_glob, "sum")
            chunk_len = auto_chunk_len(int(T_glob), G)
        D, V = int(udoc.numel()), int(vocab.numel())
        pairs = None
        if dev.type == "cuda":
            from ..ops import corpus as oc
            pairs = oc.pair_build(inv, wi.to(torch.int32).contiguous(), D, V,
                                  wt.to(torch.int32).contiguous() if use_w else None,
                                  n0=0 if dist_on else int(n_event0))
        elif dist_on:
            pairs = torch_pairs(inv, wi, V)
        corpus = build_corpus(inv, wi, D, V, i64_to_u32bits(udoc), G, chunk_len,
                              weight=wt if use_w else None, pairs=pairs if dev.type == "cuda" else None)
    with timer.stage("init"):
        model = GibbsLDA(corpus, GibbsConfig(K=K, alpha=alpha, beta=beta, seed=seed), comm=comm,
                         V_global=int(vocab.numel()))
        run = LdaRun(corpus, model, udoc, vocab, {}, pairs=pairs, route=route)
        if not train:
            return run
        if ckpt is not None and ckpt.exists():
            ckpt.restore(model)
        else:
            model.initialize()
    with timer.stage("train"):
        if on_train is not None:
            on_train()
        remaining = sweeps - model.sweeps_done
        step = eval_every if eval_every > 0 else remaining
        ck_every = ckpt.every if ckpt is not None and ckpt.every > 0 else 0
        lag = int(ldac_lag) if ldac_dir else 0
        while remaining > 0:
            n = min(step, remaining)
            if ck_every:
                n = min(n, ck_every - (model.sweeps_done % ck_every))
            if lag:
                n = min(n, lag - (model.sweeps_done % lag))
            model.sweep(n)
            remaining -= n
            mixed = model.sweeps_done > burnin
            if eval_every > 0 and model.sweeps_done % eval_every == 0 and mixed:
                ll = model.record_likelihood()
                if log:
                    log(f"sweep {model.sweeps_done} loglik {ll:.6e}")
            if ck_every and model.sweeps_done % ck_every == 0:
                ckpt.save(model)
            if lag and model.sweeps_done % lag == 0 and remaining > 0 and mixed:
                from ..io import ldac
                ldac.export_gibbs(ldac_dir, model, prefix=f"{model.sweeps_done:03d}")
    model.close()
    if not model.likelihoods or model.likelihoods[-1][0] != model.sweeps_done:
        model.record_likelihood()
    run.timings.update({"sweeps": sweeps})
    return run


@dataclass
class TorchPairs:
    """CPU counterpart of ops.corpus.PairSet (only the fields owner-side scoring reads)."""
    pair_doc: torch.Tensor
    pair_word: torch.Tensor
    tok_pair: torch.Tensor


def torch_pairs(doc_ids: torch.Tensor, word_ids: torch.Tensor, V: int) -> TorchPairs:
    u, inv = torch.unique(doc_ids.to(torch.int64) * V + word_ids.to(torch.int64), return_inverse=True)
    return TorchPairs((u // V).to(torch.int32), (u % V).to(torch.int32), inv.to(torch.int32))


@traced("oni:owner_scores")
def owner_token_scores(run: LdaRun, comm: Comm) -> torch.Tensor:
    """Data-parallel scoring (K15 with a process group): every owner scores the distinct
    (doc, word) pairs of the tokens it received with its own θ rows and the global φ, and sends
    each token's score back to the rank the token came from (the reverse of the owner routing,
    4 B per token). Returns the score of every token this rank routed, in its original order.

    This replaces an all-gather of every θ row to every rank (D_global·K·4 B per rank, 320 MB at
    the 100M-flow day) plus a per-rank pair build over the events: θ never leaves its owner. The
    per-pair dot is the same kernel as world 1 (k_pair_score), so scores stay bitwise equal."""
    ps = ops.pair_score(run.model.theta(), run.model.phi(), run.pairs.pair_doc, run.pairs.pair_word)
    return return_to_origin(ps[run.pairs.tok_pair.long()], run.route, comm)


def owner_event_scores(ts: torch.Tensor, n: int, n_sides: int, tol: float, hist: torch.Tensor,
                       want_parts: bool = False):
    """(score, s1, s2) per local event from owner-side token scores ``ts`` (tokens
    [i·n, (i+1)·n) are the events' i-th endpoints), in event order, with the fused order-key
    histogram."""
    idx = torch.arange(n_sides * n, dtype=torch.int32, device=ts.device)
    return ops.event_min(ts, idx[:n], idx[n:2 * n] if n_sides > 1 else None, tol=tol, want_parts=want_parts,
                         hist=hist)


@traced("oni:gather_theta")
def gather_theta(run: LdaRun, comm: Comm | None) -> tuple[torch.Tensor, torch.Tensor]:
    """Global (sorted doc keys, θ rows) on every rank (collective X05; local when world == 1)."""
    th = run.model.theta()
    keys = run.doc_keys64
    if comm is None or not comm.dist:
        return keys, th
    kp = comm.allgather_var(keys)
    tp = comm.allgather_var(th)
    keys = torch.cat(kp)
    th = torch.cat(tp)
    order = torch.argsort(keys)
    return keys[order].contiguous(), th[order].contiguous()


def lookup(sorted_keys: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    idx = torch.searchsorted(sorted_keys, q)
    idx = idx.clamp_(max=max(sorted_keys.numel() - 1, 0))
    if sorted_keys.numel() and not bool((sorted_keys[idx] == q).all()):
        raise KeyError("lookup key missing from dictionary")
    return idx.to(torch.int32)


@dataclass
class TilePlan:
    """16-doc × 16-word MFMA blocks covering every distinct pair (k_tile_score items)."""
    item_docs: torch.Tensor   # int32 [n_items*16] θ row of each tile row (-1: none)
    item_words: torch.Tensor  # int32 [n_items*16] φ row of each block column (-1: none)
    item_p0: torch.Tensor     # int64 [n_items+1] pair range of each item (pairs are item-major)
    pair_rc: torch.Tensor     # uint8 [P] (row << 4) | col of each pair inside its item

    @property
    def n_items(self) -> int:
        return int(self.item_p0.numel()) - 1

    def density(self) -> float:
        """Fraction of the computed 16×16 outputs that are real pairs."""
        return float(self.pair_rc.numel()) / max(256 * self.n_items, 1)


@dataclass
class ScorePlan:
    """Distinct (doc, word) pairs of a set of events + each event endpoint's pair index (K09/K15).

    Built once per day after training (the dictionaries are final); scoring is then one SDDMM
    over the distinct pairs (ops.pair_score on the VALU, or ops.tile_score on MFMA blocks when
    ``tiles`` is set; pairs are then stored item-major) and a 4-B gather per endpoint
    (ops.event_min)."""
    pdoc: torch.Tensor
    pword: torch.Tensor
    inv: list
    tiles: TilePlan | None = None
    # events regrouped by their first endpoint's pair (SCORE_SORT_EVENTS): the gather of that
    # endpoint's pair score becomes a monotone stream instead of a random 4-B read per event;
    # ``order`` maps plan position → event, ``rank`` event → plan position (built on first use:
    # the pipelines map result rows through top_n's positions and never need the full inverse)
    order: torch.Tensor | None = None
    inv_sorted: list | None = None
    _rank: torch.Tensor | None = None

    @property
    def n_pairs(self) -> int:
        return int(self.pdoc.numel())

    @property
    def rank(self) -> torch.Tensor | None:
        if self._rank is None and self.order is not None:
            order = self.order
            self._rank = torch.empty_like(order)
            self._rank[order] = torch.arange(order.numel(), dtype=order.dtype, device=order.device)
        return self._rank


def tile_plan(pdoc: torch.Tensor, pword: torch.Tensor, D: int, V: int) -> tuple[TilePlan, torch.Tensor]:
    """Group distinct pairs into MFMA items; returns (plan, perm) with pairs[perm] item-major.

    Documents are ordered heaviest first (then by their smallest word), so the dense rows of
    heavy IPs share tiles and single-pair documents with the same word share a block column.
    A tile is 16 consecutive documents of that order; its words (the union over its documents)
    are cut into blocks of 16; an item is one (tile, block).
    """
    dev = pdoc.device
    i64 = torch.int64
    P = pdoc.numel()
    pd, pw = pdoc.to(i64), pword.to(i64)
    npairs = torch.bincount(pd, minlength=D)
    first = torch.full((D,), V, dtype=i64, device=dev).scatter_reduce_(0, pd, pw, reduce="amin")
    _, o1 = torch.sort(first, stable=True)
    _, o2 = torch.sort(npairs[o1], descending=True, stable=True)
    dorder = o1[o2]
    rank = torch.empty(D, dtype=i64, device=dev)
    rank[dorder] = torch.arange(D, dtype=i64, device=dev)
    prank = rank[pd]
    tile, row = prank // 16, prank % 16
    n_tiles = (D + 15) // 16
    tile_docs = torch.full((n_tiles * 16,), -1, dtype=torch.int32, device=dev)
    tile_docs[:D] = dorder.to(torch.int32)
    u, inv = torch.unique(tile * V + pw, return_inverse=True)
    utile = u // V
    tcount = torch.bincount(utile, minlength=n_tiles)
    tstart = _excl_cumsum(tcount)
    col = torch.arange(u.numel(), dtype=i64, device=dev) - tstart[utile]
    nblk = (tcount + 15) // 16
    istart = _excl_cumsum(nblk)
    n_items = int(istart[-1])
    uitem = istart[utile] + col // 16
    item_words = torch.full((n_items * 16,), -1, dtype=torch.int32, device=dev)
    item_words[uitem * 16 + col % 16] = (u % V).to(torch.int32)
    item_tile = torch.repeat_interleave(torch.arange(n_tiles, dtype=i64, device=dev), nblk)
    item_docs = tile_docs.view(n_tiles, 16)[item_tile].reshape(-1).contiguous()
    p_item = uitem[inv]
    rc = row * 16 + (col % 16)[inv]
    perm = torch.argsort(p_item * 256 + rc)
    item_p0 = _excl_cumsum(torch.bincount(p_item, minlength=n_items))
    plan = TilePlan(item_docs, item_words, item_p0.contiguous(), rc[perm].to(torch.uint8).contiguous())
    if P != int(item_p0[-1]):
        raise AssertionError("tile plan lost pairs")
    return plan, perm


def _excl_cumsum(x: torch.Tensor) -> torch.Tensor:
    out = torch.zeros(x.numel() + 1, dtype=torch.int64, device=x.device)
    if x.numel():
        torch.cumsum(x.to(torch.int64), 0, out=out[1:])
    return out


# MFMA block scoring is kept as an option: at K = 20 and the flow day's 12 % block density the
# VALU pair dot measured 39 µs vs 74 µs for k_tile_score (profiles/r1_pmc_score_mfma_vs_valu.json)
SCORE_TILES = False
# score events in first-endpoint pair order (one monotone + one random gather per flow instead of
# two random ones; DNS/proxy events become a pure stream); results map back through plan.order
SCORE_SORT_EVENTS = True


@traced("oni:score_plan")
def score_plan(dkeys: torch.Tensor, vocab: torch.Tensor, sides, tiles: bool | None = None,
               sort_events: bool | None = None) -> ScorePlan:
    """``sides``: [(doc_keys64, word_keys64)] per event endpoint (1 for DNS/proxy, 2 for flows).

    ``tiles`` (default :data:`SCORE_TILES`) also builds the MFMA item plan and stores the pairs
    item-major."""
    V = int(vocab.numel())
    ids = [lookup(dkeys, dk).to(torch.int64) * V + lookup(vocab, wk).to(torch.int64) for dk, wk in sides]
    uniq, inv = torch.unique(torch.cat(ids), return_inverse=True)
    if uniq.numel() >= 2**31:
        raise ValueError("too many distinct pairs for int32 indices")
    pdoc, pword = uniq // V, uniq % V
    tp = None
    if SCORE_TILES if tiles is None else tiles:
        tp, perm = tile_plan(pdoc, pword, int(dkeys.numel()), V)
        newpos = torch.empty_like(perm)
        newpos[perm] = torch.arange(perm.numel(), dtype=perm.dtype, device=perm.device)
        pdoc, pword, inv = pdoc[perm], pword[perm], newpos[inv]
    invs = [x.to(torch.int32).contiguous() for x in inv.split([t.numel() for t in ids])]
    plan = ScorePlan(pdoc.to(torch.int32).contiguous(), pword.to(torch.int32).contiguous(), invs, tp)
    if SCORE_SORT_EVENTS if sort_events is None else sort_events:
        order = torch.argsort(invs[0], stable=True)
        plan.order = order
        plan.inv_sorted = [x[order].contiguous() for x in invs]
    return plan


def plan_from_pairs(ps, n: int, n_sides: int, doc_rows: torch.Tensor | None = None) -> ScorePlan:
    """Score plan straight from a pair build over the events' tokens (side-major: tokens
    [i·n, (i+1)·n) are the i-th endpoints): the distinct pairs are the SDDMM items, ``tok_pair`` is
    every endpoint's pair index and ``order0`` the first-endpoint event order -- no unique /
    searchsorted pass over the events. ``doc_rows`` maps the pair build's doc ids to θ rows."""
    pdoc = ps.pair_doc if doc_rows is None else doc_rows[ps.pair_doc.long()].to(torch.int32)
    invs = [ps.tok_pair[i * n:(i + 1) * n] for i in range(n_sides)]
    plan = ScorePlan(pdoc.contiguous(), ps.pair_word, invs)
    if SCORE_SORT_EVENTS and ps.order0 is not None:
        plan.order = ps.order0
        plan.inv_sorted = [x[ps.order0].contiguous() for x in invs]
    return plan


@traced("oni:score_plan")
def event_score_plan(run: LdaRun, dkeys: torch.Tensor, vocab: torch.Tensor, doc_sides: list, word_ids_ev: torch.Tensor,
                     word_sides: list, comm: Comm | None) -> ScorePlan:
    """Score plan of this rank's events (``doc_sides``: doc keys per endpoint, ``word_ids_ev``: the
    endpoints' word ids, side-major). GPU, world 1: the corpus pair build already holds it. GPU with
    a process group: a local pair build over the events (owner routing moved the corpus tokens
    away), its doc ids mapped to rows of the gathered θ (``dkeys``) through the local unique docs
    only. CPU: the torch reference :func:`score_plan`."""
    n = int(doc_sides[0].numel())
    if not doc_sides[0].is_cuda or SCORE_TILES:
        return score_plan(dkeys, vocab, list(zip(doc_sides, word_sides)))
    if run.pairs is not None:
        return plan_from_pairs(run.pairs, n, len(doc_sides))
    from ..ops import corpus as oc
    ludoc, lids = encode_docs(torch.cat(doc_sides) if len(doc_sides) > 1 else doc_sides[0].contiguous())
    eps = oc.pair_build(lids, word_ids_ev.to(torch.int32).contiguous(), int(ludoc.numel()), int(vocab.numel()), n0=n)
    return plan_from_pairs(eps, n, len(doc_sides), doc_rows=lookup(dkeys, ludoc))


@traced("oni:score")
def plan_score(theta: torch.Tensor, phi: torch.Tensor, plan: ScorePlan, tol: float, hist=None, want_parts=False):
    """(score, s1, s2) per event in PLAN order (event order unless plan.order is set; map plan
    positions back with plan.order / event indices forward with plan.rank)."""
    if plan.tiles is not None:
        t = plan.tiles
        ps = ops.tile_score(theta, phi, t.item_docs, t.item_words, t.item_p0, t.pair_rc, plan.pdoc, plan.pword)
    else:
        ps = ops.pair_score(theta, phi, plan.pdoc, plan.pword)
    inv = plan.inv_sorted if plan.inv_sorted is not None else plan.inv
    return ops.event_min(ps, inv[0], inv[1] if len(inv) > 1 else None, tol=tol, want_parts=want_parts, hist=hist)


def to_event_order(plan: ScorePlan, x: torch.Tensor | None) -> torch.Tensor | None:
    """Per-event values produced in plan order (plan_score) → event order."""
    if x is None or plan.rank is None:
        return x
    return x[plan.rank]


@traced("oni:top_n")
def top_n(score: torch.Tensor, tol: float, maxresults: int, comm: Comm | None, row_offset: int = 0,
          hist: torch.Tensor | None = None, order: torch.Tensor | None = None, return_pos: bool = False):
    """Lowest ``maxresults`` scores below ``tol`` (ties by global row id), merged over ranks (X06).

    ``hist`` is the 2048-bucket histogram of score order keys (top 11 bits) of events under tol,
    as produced by the fused score kernel; computed here when absent. Returns (global row ids
    int64, scores f32), ascending, identical on every rank. ``order`` (a score plan's event order)
    maps positions of ``score`` to local event ids. ``return_pos`` (no process group) also returns
    each result row's position in ``score``.
    """
    if hist is None:
        b = u32_to_i64(ops.f32_keys(score)) >> 21
        hist = torch.bincount(b[score < tol], minlength=2048)
    return _top_n_from_hist(score, hist, tol, maxresults, comm, row_offset, order, return_pos)


@dataclass
class SingleResult:
    rows: np.ndarray      # global row ids, ascending score
    scores: np.ndarray
    words: np.ndarray     # packed word keys (u64) of the result rows
    timings: dict
    stats: dict
    lda: object = None


def run_single_doc_events(doc_keys64: torch.Tensor, word_keys64: torch.Tensor, K: int, sweeps: int, tol: float,
                          maxresults: int, alpha, beta: float, seed: int, chunk_len: int, comm: Comm | None,
                          feedback=None, row_offset: int = 0, eval_every: int = 0, burnin: int = 0, ckpt=None, log=None,
                          timer: StageTimer | None = None, ldac_dir: str | None = None,
                          ldac_lag: int = 0, key_bits: int = 64) -> SingleResult:
    """Shared DNS/proxy path: one (doc, word) token per event; score = θ_doc·φ_word (C24)."""
    dev = doc_keys64.device
    timer = timer or StageTimer(dev)
    with timer.stage("vocab"):
        dk, wk, wts = doc_keys64, word_keys64, None
        if feedback is not None:
            wts = torch.cat([torch.ones_like(wk), feedback[2]]).to(torch.int32)
            dk = torch.cat([dk, feedback[0]])
            wk = torch.cat([wk, feedback[1]])
        vocab, wids = encode_words(wk.contiguous(), comm, key_bits)
    n = int(doc_keys64.numel())
    run = build_and_train(dk, None, wts, vocab, K, alpha, beta, seed, sweeps, chunk_len, comm, eval_every=eval_every, burnin=burnin,
                          ckpt=ckpt, log=log, timer=timer, ldac_dir=ldac_dir, ldac_lag=ldac_lag, word_ids=wids,
                          n_event0=n)
    hist = torch.zeros(2048, dtype=torch.int32, device=dev)
    if run.route is not None:
        with timer.stage("score_prep"):
            ts = owner_token_scores(run, comm)
        with timer.stage("score"):
            score, _, _ = owner_event_scores(ts, n, 1, tol, hist)
            rows, scs = top_n(score, tol, maxresults, comm, row_offset, hist=hist)
    else:
        with timer.stage("score_prep"):
            dkeys, theta = gather_theta(run, comm)
            plan = event_score_plan(run, dkeys, vocab, [doc_keys64], wids[:n], [word_keys64], comm)
        with timer.stage("score"):
            score, _, _ = plan_score(theta, run.model.phi(), plan, tol, hist=hist)
            rows, scs = top_n(score, tol, maxresults, comm, row_offset, hist=hist, order=plan.order)
    t = timer.summary()
    t.update(run.timings)
    t["records_scored"] = int(doc_keys64.numel())
    loc = rows - row_offset
    mine = (loc >= 0) & (loc < doc_keys64.numel())
    words = word_keys64[loc[mine]]
    if comm is not None and comm.dist:
        allp = torch.cat(comm.allgather_var(torch.stack([rows[mine].to(torch.int64), words.to(torch.int64)], 1))).cpu()
        words = allp[rows_in_order(allp[:, 0], rows.cpu()), 1]
    stats = run.corpus.stats()
    stats.update({"events": int(doc_keys64.numel()),
                  "loglik": run.model.likelihoods[-1][1] if run.model.likelihoods else None})
    return SingleResult(rows=rows.cpu().numpy(), scores=scs.cpu().numpy(),
                        words=words.cpu().numpy().view(np.uint64), timings=t, stats=stats, lda=run)


def rows_in_order(gid_all: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    """Index of every id of ``rows`` in ``gid_all`` (a permutation of the same distinct ids)."""
    o = torch.argsort(gid_all)
    return o[torch.searchsorted(gid_all[o], rows)]


def _top_n_from_hist(score, hist, tol, maxresults, comm, row_offset, order=None, return_pos=False):
    h_loc = hist.to(torch.int64).cpu().numpy()
    h = comm.allreduce_np(h_loc) if comm is not None and comm.dist else h_loc
    cum = np.cumsum(h)
    if maxresults <= 0 or cum[-1] == 0:
        bmax = 2047 if maxresults > 0 else -1
    else:
        bmax = int(np.searchsorted(cum, min(maxresults, int(cum[-1])), side="left"))
    if return_pos and comm is not None and comm.dist:
        raise ValueError("top_n: positions are only defined without a process group")
    if bmax < 0:
        e = torch.zeros(0, dtype=torch.int64, device=score.device)
        out = (e, torch.zeros(0, dtype=torch.float32, device=score.device))
        return out + (e,) if return_pos else out
    # the local histogram already counts this rank's candidates: no extra pass over the scores
    cap = int(np.cumsum(h_loc)[bmax])
    pos, sc = ops.select_below(score, tol, bmax, cap=max(cap, 1))
    idx = order[pos] if order is not None else pos
    gid = idx + row_offset
    # exact order: (score, global id); keep local top-N then merge
    o1 = torch.argsort(gid, stable=True)
    o2 = o1[torch.argsort(sc[o1], stable=True)][:maxresults]
    gid, sc = gid[o2], sc[o2]
    if return_pos:
        return gid, sc, pos[o2]
    if comm is not None and comm.dist:
        # one all-gather of (global id, score bits) pairs
        both = torch.cat(comm.allgather_var(torch.stack([gid.to(torch.int64),
                                                         sc.view(torch.int32).to(torch.int64)], 1)))
        gid, sc = both[:, 0].contiguous(), both[:, 1].to(torch.int32).view(torch.float32)
        o1 = torch.argsort(gid, stable=True)
        gid, sc = gid[o1], sc[o1]
        o2 = torch.argsort(sc, stable=True)
        gid, sc = gid[o2][:maxresults], sc[o2][:maxresults]
    return gid, sc
