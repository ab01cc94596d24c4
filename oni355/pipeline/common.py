"""Source-independent stages of suspicious-connects: vocabulary, owner routing, corpus, LDA,
scoring and top-N selection (the oni-ml pre-LDA / LDA / post-LDA skeleton).

Data-parallel layout: every rank featurizes its own events; tokens are
routed to the rank that owns their document (hash of the document key), so each rank's corpus is
document-complete and the sampler needs only the per-sweep Δn_wk all-reduce. Word ids come from
one global sorted vocabulary (all-gather of local unique keys, X02), so ids -- and therefore every
sample -- are independent of the GPU count.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..ref import spec
from ..utils.obs import StageTimer, traced
from ..models.corpus import Corpus, auto_chunk_len, build_corpus
from ..models.gibbs import GibbsConfig, GibbsLDA
from ..parallel.comm import Comm

U32MASK = 0xFFFFFFFF


class DayCuts:
    """A day's quantile cut lists by feature name, computed on the device
    (:func:`ops.quantile_cuts_dev`): kernels take ``dev`` (the lists concatenated, int32 bits);
    the host arrays are fetched on first access (one copy)."""

    def __init__(self, names: list, sizes: list, dev: torch.Tensor):
        self.names, self.sizes, self.dev = list(names), [int(x) for x in sizes], dev
        self._host = None

    def _h(self) -> dict:
        if self._host is None:
            a = self.dev.cpu().numpy().view(np.uint32)
            off = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
            self._host = {n: a[off[i]:off[i + 1]].copy() for i, n in enumerate(self.names)}
        return self._host

    def __getitem__(self, k):
        return self._h()[k]

    def items(self):
        return self._h().items()

    def keys(self):
        return list(self.names)


def binned_cuts(keys: dict, binned: list, comm: Comm | None, n_glob: int):
    """Quantile cuts of the BINNED features of a DNS / proxy day: on a GPU the radix select and
    the digit picks stay on the stream (:class:`DayCuts`); on the CPU the oracle path. Returns
    (cuts, device concatenation or None)."""
    names = [name for name, _, _ in binned]
    fr = [f for _, f, _ in binned]
    kl = [keys[name].contiguous() for name in names]
    if kl[0].is_cuda:
        dev_ar = comm.allreduce_ if comm is not None and comm.dist else None
        dc = ops.quantile_cuts_dev(kl, fr, dev_ar, n_glob)
        return DayCuts(names, [len(f) for f in fr], dc), dc
    ar = comm.allreduce_np if comm is not None and comm.dist else None
    return dict(zip(names, ops.quantile_cuts_multi(kl, fr, ar, n_glob))), None


def u32_to_i64(t: torch.Tensor) -> torch.Tensor:
    """int32 tensor holding u32 bits → non-negative int64."""
    return t.to(torch.int64) & U32MASK


def i64_to_u32bits(t: torch.Tensor) -> torch.Tensor:
    return (t & U32MASK).to(torch.int64).to(torch.int32) if t.dtype == torch.int64 else t


def feedback_here(comm: Comm | None) -> bool:
    """Does this rank contribute the analyst feedback tokens (C19)? Every rank reads the same
    scores CSV, but its sev = 3 rows must enter the GLOBAL corpus once -- DUPFACTOR times, not
    world × DUPFACTOR -- so only rank 0 adds them; owner routing then sends each token to the rank
    that owns its document, and the corpus equals the single-GPU one."""
    return comm is None or not comm.dist or comm.rank == 0


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
    if comm is None or not comm.live:
        return luniq, lids  # one rank: the local dictionary is the global one
    parts = comm.allgather_var(luniq)
    vocab = torch.unique(torch.cat([p.to(luniq.device) for p in parts]))
    remap = torch.searchsorted(vocab, luniq).to(torch.int32)
    return vocab, remap[lids.long()]


@traced("oni:global_vocab")
def global_vocab(keys64: torch.Tensor, comm: Comm | None) -> torch.Tensor:
    """Sorted unique int64 word keys over all ranks (collective X02)."""
    return encode_words(keys64, comm)[0]


@traced("oni:encode_docs")
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


HEAVY_DOCS_PER_RANK = int(os.environ.get("ONI_HEAVY_DOCS_PER_RANK", "4096"))
PLACEMENT_BUCKETS_PER_RANK = 64
# A document holding more than 1/(SPLIT_DEN · world) of the day's tokens (one NAT gateway or
# resolver) is cut into chunk-aligned pieces that are placed like documents;
# ONI_SPLIT_DEN=0 places every document whole.
SPLIT_DEN = float(os.environ.get("ONI_SPLIT_DEN", "2"))
# smallest world that splits (tests set 1 to run the piece machinery on a forced 1-rank group)
SPLIT_MIN_WORLD = int(os.environ.get("ONI_SPLIT_MIN_WORLD", "2"))


@dataclass
class SplitPlan:
    """Heavy documents cut across ranks. Piece k of document j covers canonical token positions
    [p0, p1) of j (multiples of the chunk length L, so every piece is a run of whole chunks of the
    single-GPU layout); pieces are sampled where they are placed, against the sweep-start n_dk row
    of the whole document, and their Δn_dk rows ride in the X01 all-reduce (models/gibbs.py).
    The primary (owner of piece 0) receives all of the document's tokens for scoring and holds its
    θ row like any owned document."""
    keys: torch.Tensor        # int64 [n] doc keys of the split documents (ascending)
    count: np.ndarray         # int64 [n] global token count of each
    piece_doc: np.ndarray     # int64 [m] split index of each piece
    piece_p0: np.ndarray      # int64 [m]
    piece_p1: np.ndarray      # int64 [m]
    piece_owner: np.ndarray   # int64 [m]
    primary: np.ndarray       # int64 [n]
    L: int

    @property
    def n(self) -> int:
        return int(self.keys.numel())


def _split_pieces(counts: np.ndarray, thr: float, L: int):
    """(doc index, p0, p1) of the pieces of every count above ``thr``: runs of ⌊thr / L⌋ chunks."""
    pc = max(1, int(thr // L))
    doc, p0, p1 = [], [], []
    for i, c in enumerate(counts.tolist()):
        n_ch = -(-int(c) // L)
        for k in range(0, n_ch, pc):
            doc.append(i)
            p0.append(k * L)
            p1.append(min((k + pc) * L, int(c)))
    return np.asarray(doc, np.int64), np.asarray(p0, np.int64), np.asarray(p1, np.int64)


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


@traced("oni:place_docs")
def place_docs(doc_keys64: torch.Tensor, weights: torch.Tensor | None, comm: Comm, per_doc: bool = False,
               split_L: int | None = None):
    """Owner rank of each token's document, balanced by global token counts.

    IP documents are power-law sized (one synthetic 100M-flow day puts ~8 % of all tokens on a
    single IP), so a plain hash leaves the busiest rank ~1.5× the mean at 8 ranks and every sweep
    waits for it. Every rank proposes the documents holding more than 1/``HEAVY_DOCS_PER_RANK`` of
    its tokens (at most that many: a threshold, no sort; any document above 1/H of the global
    tokens is proposed by at least one rank); the union of the proposals gets exact global counts
    (one all-reduce over the candidates, not an all-gather of every document); every other
    document falls into one of
    ``PLACEMENT_BUCKETS_PER_RANK × world`` hash buckets, and candidates and buckets together are
    placed by longest-processing-time greedy (:func:`lpt_place`). Collective volume is
    O(candidates · world), independent of the number of documents.
    The candidate counts and bucket loads come from one kernel (``ops.corpus.place_stats``), the
    owner of every document from another (``place_owner``); the host only runs the LPT over
    ≤ H·world + 64·world items. Deterministic on every rank (same candidate set and counts; order
    count desc, key asc; ties → lowest rank); results stay world-size invariant because the
    sampler's chain never depends on placement. Returns the owner of every token, or with ``per_doc`` (owner of every local
    document int32, document id of every token int32, sorted unique local doc keys int64).
    ``split_L`` > 0 (the chunk length) also cuts candidates above 1/(SPLIT_DEN · world) of all
    tokens into pieces (:class:`SplitPlan`, appended to the return value; a split document's
    tokens go to its primary)."""
    W = comm.world
    dev = doc_keys64.device
    cuda = doc_keys64.is_cuda
    if cuda:
        from ..ops import corpus as oc
    if W == 1 and not (split_L and split_L > 0 and W >= SPLIT_MIN_WORLD and SPLIT_DEN > 0):
        # a 1-rank group owns every document (LPT puts every item on rank 0; nothing is split):
        # no counts, candidates, collectives or host round trip
        ukeys, inv = encode_docs(doc_keys64.contiguous())
        uown = torch.zeros(ukeys.numel(), dtype=torch.int32, device=dev)
        out = (uown, inv, ukeys) if per_doc else uown.long()[inv.long()]
        return (out, None) if split_L is not None else out
    if cuda:
        ukeys, inv, ucnt = oc.dict_encode(doc_keys64.contiguous(), 32,
                                          weights.to(torch.int32) if weights is not None else None, counts=True)
    else:
        ukeys, inv = encode_docs(doc_keys64.contiguous())
        w = weights.to(torch.int64) if weights is not None else torch.ones(inv.numel(), dtype=torch.int64)
        ucnt = torch.zeros(ukeys.numel(), dtype=torch.int64).index_add_(0, inv.long(), w)
    # local proposals: every document holding more than 1/H of this rank's tokens -- at most H of
    # them, picked by a threshold instead of a sort; ukeys is ascending, so the proposals are too.
    # With splitting on, also every document holding more than 1/(SPLIT_DEN · W²) of the day's
    # tokens here (≤ SPLIT_DEN · W² of them): a document above the split threshold has at least
    # 1/W of its tokens on some rank, so it is proposed whatever H, W and the shard sizes are
    splitting = bool(split_L and split_L > 0 and W >= SPLIT_MIN_WORLD and SPLIT_DEN > 0)
    heavy = ucnt * HEAVY_DOCS_PER_RANK > ucnt.sum()
    if splitting:
        total = comm.allreduce_scalar(float(ucnt.sum()))
        heavy = heavy | (ucnt.to(torch.float64) * (SPLIT_DEN * W * W) > total)
    prop = ukeys[heavy].contiguous()
    cand = prop if W == 1 else torch.unique(torch.cat([p.to(dev) for p in comm.allgather_var(prop)]))
    # all other documents are hashed into B buckets that are placed like documents, so the rank
    # that takes a huge IP takes correspondingly fewer light ones
    B = PLACEMENT_BUCKETS_PER_RANK * W
    # candidate counts ‖ bucket loads, summed over the ranks in one collective
    both = oc.place_stats(ukeys, ucnt, cand, B) if cuda else _place_stats_ref(ukeys, ucnt, cand, B)
    comm.allreduce_(both)
    nc = int(cand.numel())
    bc = both.cpu().numpy().astype(np.int64)
    ccg, bl = bc[:nc], bc[nc:]
    sp = np.zeros(nc, bool)
    if splitting:
        thr = float(bc.sum()) / (SPLIT_DEN * W)
        sp = ccg > max(thr, 2.0 * split_L)
    pdoc, pp0, pp1 = _split_pieces(ccg[sp], float(bc.sum()) / (SPLIT_DEN * W) if sp.any() else 1.0, max(split_L or 1, 1))
    ns_idx = np.nonzero(~sp)[0]
    # items in placement order: whole candidates (by key), pieces, buckets; LPT by count desc, stable
    items = np.concatenate([ccg[ns_idx], pp1 - pp0, bl])
    o = np.argsort(-items, kind="stable")
    assign = lpt_place(items[o], np.zeros(W, dtype=np.int64))
    iown = np.empty(items.size, np.int64)
    iown[o] = assign
    n_ns, n_p = ns_idx.size, pdoc.size
    cown = np.empty(nc, np.int64)
    cown[ns_idx] = iown[:n_ns]
    piece_owner = iown[n_ns:n_ns + n_p]
    sp_idx = np.nonzero(sp)[0]
    primary = np.empty(sp_idx.size, np.int64)
    if n_p:
        first = np.r_[True, pdoc[1:] != pdoc[:-1]]
        primary[:] = piece_owner[first]
        cown[sp_idx] = primary
    bown = torch.from_numpy(iown[n_ns + n_p:].astype(np.int32)).to(dev)
    cown_t = torch.from_numpy(cown.astype(np.int32)).to(dev)
    uown = oc.place_owner(ukeys, cand, cown_t, bown) if cuda else _place_owner_ref(ukeys, cand, cown_t, bown)
    plan = None
    if sp.any():
        plan = SplitPlan(keys=cand[torch.from_numpy(sp_idx).to(dev)].cpu(), count=ccg[sp], piece_doc=pdoc,
                         piece_p0=pp0, piece_p1=pp1, piece_owner=piece_owner, primary=primary, L=int(split_L))
    if per_doc:
        out = (uown, inv, ukeys)
    else:
        out = uown.long()[inv.long()]
    return (out, plan) if split_L is not None else out


def _place_stats_ref(ukeys: torch.Tensor, ucnt: torch.Tensor, cand: torch.Tensor, B: int) -> torch.Tensor:
    """Torch twin of ``ops.corpus.place_stats`` (the CPU path): candidate counts ‖ bucket loads."""
    nc = int(cand.numel())
    both = torch.zeros(nc + B, dtype=torch.int64, device=ukeys.device)
    hit = torch.zeros(ukeys.numel(), dtype=torch.bool, device=ukeys.device)
    if nc and ukeys.numel():
        pos = torch.searchsorted(cand, ukeys).clamp_(max=nc - 1)
        hit = cand[pos] == ukeys
        both[pos[hit]] = ucnt[hit]
    both[nc:].index_add_(0, doc_owner(ukeys[~hit], B), ucnt[~hit])
    return both


def _place_owner_ref(ukeys: torch.Tensor, cand: torch.Tensor, cown: torch.Tensor, bown: torch.Tensor) -> torch.Tensor:
    """Torch twin of ``ops.corpus.place_owner``: owner of every document (int32)."""
    uown = bown[doc_owner(ukeys, int(bown.numel()))]
    nc = int(cand.numel())
    if nc and ukeys.numel():
        pos = torch.searchsorted(cand, ukeys).clamp_(max=nc - 1)
        hit = cand[pos] == ukeys
        uown[hit] = cown[pos[hit]]
    return uown


def balanced_owner(doc_keys64: torch.Tensor, weights: torch.Tensor, comm: Comm) -> torch.Tensor:
    """Alias of :func:`place_docs` (round-1 name)."""
    return place_docs(doc_keys64, weights, comm)


@dataclass
class Route:
    """How this rank's tokens were sent to their document owners (for the way back)."""
    order: torch.Tensor     # int [n_sent]: slot i of the owner-grouped send buffer holds token order[i]
    send_counts: list       # tokens sent to each rank
    recv_counts: list       # tokens received from each rank (the owner side's layout)
    split: SplitPlan | None = None  # heavy documents cut across ranks (their tokens went to the primary)


@traced("oni:route_to_owners")
def route_to_owners(doc_keys64: torch.Tensor, word_ids: torch.Tensor, weights: torch.Tensor | None,
                    comm: Comm | None, split_L: int = 0):
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
        (uown, ids, ukeys), plan = place_docs(doc_keys64, weights, comm, per_doc=True, split_L=split_L)
        W = comm.world
        # key lists per owner (the local docs grouped by owner, ascending keys inside a group) and
        # every doc's position in its owner's list: one stable partition of the documents
        _, kcounts, pos, ksend = oc.partition(uown, W, keys64=ukeys, rank=True)
        send, order, counts = oc.route_pack_ids(uown, ids, pos, word_ids.to(torch.int32).contiguous(),
                                                weights, W)
        # both count vectors travel in one small exchange, then the two payload alltoallvs; one
        # host read for sent and received counts
        sc = torch.stack([counts, kcounts], 1).reshape(-1).contiguous()
        rcm = comm.alltoallv(sc.view(W, 2), [1] * W, recv_counts=[1] * W).reshape(-1)
        host = torch.cat([sc, rcm.to(sc.device)]).tolist()
        scl, kcl, rc, krc = host[0:2 * W:2], host[1:2 * W:2], host[2 * W::2], host[2 * W + 1::2]
        rkeys = comm.alltoallv(ksend, kcl, recv_counts=krc)
        recv = comm.alltoallv(send, scl, recv_counts=rc)
        if W == 1:
            # a 1-rank group receives its own ascending key list: it already is the dictionary
            udoc = ukeys
            kid = torch.arange(udoc.numel(), dtype=torch.int32, device=udoc.device)
        else:
            udoc, kid = encode_docs(u32_to_i64(rkeys.view(-1)).contiguous())
        inv, wi, wt = oc.route_unpack(recv.contiguous(), rc, krc, kid, weights is not None)
        return udoc, inv, wi, wt, Route(order, scl, rc, plan)
    owner, plan = place_docs(doc_keys64, weights, comm, split_L=split_L)
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
    return udoc, inv, wi, wt, Route(order, counts.tolist(), rc, plan)


@traced("oni:return_to_origin")
def return_to_origin(x: torch.Tensor, route: Route, comm: Comm) -> torch.Tensor:
    """Inverse of :func:`route_to_owners` for a per-received-token value ``x`` (owner layout):
    returns the value of every token this rank sent, in its original token order."""
    back = comm.alltoallv(x.contiguous(), route.recv_counts, recv_counts=route.send_counts)
    out = torch.empty_like(back)
    out[route.order.to(back.device).long()] = back
    return out


def split_corpus_tokens(plan: SplitPlan, udoc: torch.Tensor, inv: torch.Tensor, wi: torch.Tensor, wt: torch.Tensor,
                        V: int, comm: Comm):
    """Corpus token list of this rank with the split documents replaced by the pieces it was
    assigned: (doc id int32, word id int32, weight int32, doc keys int64 [D_own + pieces], meta).

    Each split document's primary contributes the document's (word, Σ weight) pairs (one
    all-gather of ≤ V pairs per split document); every rank then expands the canonical order of
    the documents it holds pieces of (pairs by word id, as :mod:`oni355.models.corpus` orders a
    document) and clips it to each piece's [p0, p1): piece pairs enter the corpus as weighted
    tokens of new rows D_own, D_own + 1, ... The primary's own row keeps the document's θ and
    samples nothing."""
    dev = inv.device
    i64 = torch.int64
    D_own = int(udoc.numel())
    skeys = plan.keys.to(dev)
    n = plan.n
    row_j = torch.full((max(D_own, 1),), -1, dtype=i64, device=dev)
    if D_own:
        pos = torch.searchsorted(udoc, skeys).clamp_(max=D_own - 1)
        hit = udoc[pos] == skeys
        row_j[pos[hit]] = torch.arange(n, device=dev)[hit]
    prim = torch.nonzero(row_j[:D_own] >= 0).flatten()
    tokj = row_j[inv.long()] if inv.numel() else torch.zeros(0, dtype=i64, device=dev)
    m = tokj >= 0
    key = tokj[m] * V + wi[m].to(i64)
    u, ui = torch.unique(key, return_inverse=True)
    cnt = torch.zeros(u.numel(), dtype=i64, device=dev).index_add_(0, ui, wt[m].to(i64))
    rows = torch.stack([u // V, u % V, cnt], 1).contiguous()
    allp = torch.cat([p.to(dev) for p in comm.allgather_var(rows)]) if comm.live else rows
    allp = allp[torch.argsort(allp[:, 0] * V + allp[:, 1])]
    mine = np.nonzero(plan.piece_owner == comm.rank)[0]
    pd, pw, pc = [], [], []
    for t, k in enumerate(mine.tolist()):
        pj = allp[allp[:, 0] == int(plan.piece_doc[k])]
        e = torch.cumsum(pj[:, 2], 0)
        ov = torch.clamp(torch.minimum(e, torch.tensor(int(plan.piece_p1[k]), device=dev))
                         - torch.maximum(e - pj[:, 2], torch.tensor(int(plan.piece_p0[k]), device=dev)), min=0)
        keep = ov > 0
        pw.append(pj[keep, 1])
        pc.append(ov[keep])
        pd.append(torch.full((int(keep.sum()),), D_own + t, dtype=i64, device=dev))
    keep_tok = ~m
    z = torch.zeros(0, dtype=i64, device=dev)
    tdoc = torch.cat([inv[keep_tok].to(i64), *pd, z]).to(torch.int32).contiguous()
    tword = torch.cat([wi[keep_tok].to(i64), *pw, z]).to(torch.int32).contiguous()
    twt = torch.cat([wt[keep_tok].to(i64), *pc, z]).to(torch.int32).contiguous()
    pj_idx = torch.from_numpy(plan.piece_doc[mine]).to(dev)
    dkeys = torch.cat([udoc, skeys[pj_idx]]) if mine.size else udoc
    piece_tokens = int(sum(int(x.sum()) for x in pc))
    meta = dict(D_own=D_own, n_split=n, piece_rows=torch.arange(D_own, D_own + mine.size, device=dev),
                piece_j=pj_idx, piece_p0=torch.from_numpy(plan.piece_p0[mine]).to(dev), prim_rows=prim,
                prim_j=row_j[prim], piece_tokens=piece_tokens,
                prim_tokens=int(plan.count[row_j[prim].cpu().numpy()].sum()) if prim.numel() else 0,
                max_count=int(plan.count.max()) if n else 0)
    return tdoc, tword, twt, dkeys, meta


def apply_split(corpus: Corpus, meta: dict) -> None:
    """Attach the split metadata to a corpus built from :func:`split_corpus_tokens`: piece rows
    sample like chunks of a long document (sweep-start row snapshot + atomic Δ into a seeded
    copy), and their chunks draw from the document's GLOBAL canonical positions (Philox counter)."""
    dev = corpus.chunk_doc.device
    D = corpus.D
    pos0 = torch.zeros(max(D, 1), dtype=torch.int64, device=dev)
    is_piece = torch.zeros(max(D, 1), dtype=torch.bool, device=dev)
    pr = meta["piece_rows"]
    pos0[pr] = meta["piece_p0"]
    is_piece[pr] = True
    cd = corpus.chunk_doc.to(torch.int64)
    live = cd >= 0
    cdl = cd.clamp(min=0)
    corpus.chunk_multi = (corpus.chunk_multi.bool() | (live & is_piece[cdl])).to(torch.uint8)
    corpus.chunk_rng0 = torch.where(live, corpus.chunk_pos0.to(torch.int64) + pos0[cdl],
                                    corpus.chunk_pos0.to(torch.int64)).to(torch.int32).contiguous()
    corpus.long_rows = torch.unique(torch.cat([corpus.long_rows.to(torch.int64), pr])).to(torch.int32)
    meta["doc_pos0"] = pos0[:D]
    meta["own_tokens"] = corpus.T - meta["piece_tokens"] + meta["prim_tokens"]
    corpus.split = meta


@dataclass
class ChainEstimate:
    """θ and φ of a finished extra chain (ONI_CHAINS > 1): all that scoring reads of it."""
    theta_rows: torch.Tensor
    phi_rows: torch.Tensor
    sweeps_done: int

    def theta(self) -> torch.Tensor:
        return self.theta_rows

    def phi(self) -> torch.Tensor:
        return self.phi_rows


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
    # independent chains beyond ``model`` (ONI_CHAINS > 1): scores are averaged over all chains
    extra_models: list = field(default_factory=list)

    def pair_scores(self, theta: torch.Tensor, phi: torch.Tensor, pdoc: torch.Tensor,
                    pword: torch.Tensor) -> torch.Tensor:
        """θ·φ of every (doc, word) pair, averaged in score space over the chains (θ / φ of the
        first chain given; topic labels differ between chains, so only scores can be averaged)."""
        ps = ops.pair_score(theta, phi, pdoc, pword)
        if not self.extra_models:
            return ps
        D = theta.shape[0]
        for m in self.extra_models:
            ps = ps + ops.pair_score(m.theta()[:D], m.phi(), pdoc, pword)
        return ps * np.float32(1.0 / (1 + len(self.extra_models)))


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
        from ..models.gibbs import mh_burn_for, sampler_for, tiling_for
        G, _ = tiling_for(K)
        mh = sampler_for(K) == "mh"
        # an MH model's first sweeps run the dense kernel on a corpus of the dense tiling
        burn_mh = mh_burn_for(sweeps) if mh and train else 0
        Gd = tiling_for(K, "dense")[0] if burn_mh else G
        if chunk_len <= 0:
            # the global (weighted) token count picks L -- before routing: the placement cuts
            # heavy documents at multiples of L
            T_glob = float(weights.sum()) if use_w else float(doc_keys64.numel())
            if dist_on:
                T_glob = comm.allreduce_scalar(T_glob, "sum")
            # the MH sampler's u8 LDS cells hold a chunk's count deltas: chunks ≤ 127 tokens
            chunk_len = auto_chunk_len(int(T_glob), G, hi=spec.MH_MAX_CHUNK if mh else 128)
        elif mh and chunk_len > spec.MH_MAX_CHUNK:
            # an explicit CHUNK_LEN (valid up to 128 for the dense kernels) above the MH sampler's
            # limit: clamp rather than fail the day
            if log:
                log(f"chunk_len {chunk_len} -> {spec.MH_MAX_CHUNK}: the MH sampler's chunks hold at most "
                    f"{spec.MH_MAX_CHUNK} tokens")
            chunk_len = spec.MH_MAX_CHUNK
        udoc, inv, wi, wt, route = route_to_owners(doc_keys64, word_ids, weights, comm,
                                                   split_L=chunk_len if dist_on else 0)
        D, V = int(udoc.numel()), int(vocab.numel())
        pairs = None
        if dev.type == "cuda":
            from ..ops import corpus as oc
            pairs = oc.pair_build(inv, wi.to(torch.int32).contiguous(), D, V,
                                  wt.to(torch.int32).contiguous() if use_w else None,
                                  n0=0 if dist_on else int(n_event0))
        elif dist_on:
            pairs = torch_pairs(inv, wi, V)
        plan = route.split if route is not None else None
        if plan is not None:
            # heavy documents cut across ranks: the corpus holds this rank's pieces (pairs clipped
            # to their canonical ranges) instead of the tokens the primary received for scoring
            tdoc, tword, twt, dkeys, meta = split_corpus_tokens(plan, udoc, inv, wi, wt, V, comm)

            def corpus_for(g):
                c = build_corpus(tdoc, tword, int(dkeys.numel()), V, i64_to_u32bits(dkeys), g, chunk_len, weight=twt)
                apply_split(c, meta)
                return c
        else:
            def corpus_for(g):
                return build_corpus(inv, wi, D, V, i64_to_u32bits(udoc), g, chunk_len,
                                    weight=wt if use_w else None, pairs=pairs if dev.type == "cuda" else None)
        corpus = corpus_for(G)
        dcorpus = corpus_for(Gd) if Gd != G else None
    # ONI_CHAINS = C > 1: C independent chains of sweeps // C sweeps each (same total sweep count),
    # scored by the average of their pair scores (LdaRun.pair_scores): the top-N then depends less
    # on any one chain's seed. Dense samplers only, no checkpointing.
    chains = max(1, int(os.environ.get("ONI_CHAINS", "1")))
    if chains > 1 and (mh or ckpt is not None or not train or sweeps < 2 * chains):
        chains = 1
    if chains > 1:
        sweeps = sweeps // chains
    with timer.stage("init"):
        model = GibbsLDA(corpus, GibbsConfig(K=K, alpha=alpha, beta=beta, seed=seed), comm=comm,
                         V_global=int(vocab.numel()))
        run = LdaRun(corpus, model, udoc, vocab, {}, pairs=pairs, route=route)
        if not train:
            return run
        model.plan_average(sweeps)
        win = model.average_window
        if win is not None and dcorpus is not None:
            burn_mh = min(burn_mh, win[0] - 1)  # the MH model takes every posterior sample
        burner = None  # the dense model of an MH model's first burn_mh sweeps
        if burn_mh <= 0:
            dcorpus = None
        if mh:
            model.chain["mh_burn"] = burn_mh if dcorpus is not None else 0
        if dcorpus is not None and not (ckpt is not None and ckpt.exists() and ckpt.manifest()["sweep"] >= burn_mh):
            burner = GibbsLDA(dcorpus, GibbsConfig(K=K, alpha=alpha, beta=beta, seed=seed, sampler="dense"),
                              comm=comm, V_global=int(vocab.numel()))
            burner.chain = model.chain  # its checkpoints belong to the MH run
        first = burner or model
        if ckpt is not None and ckpt.exists():
            ckpt.restore(first)
        else:
            first.initialize()
    with timer.stage("train"):
        if on_train is not None:
            on_train()
        remaining = sweeps - first.sweeps_done
        step = eval_every if eval_every > 0 else remaining
        ck_every = ckpt.every if ckpt is not None and ckpt.every > 0 else 0
        lag = int(ldac_lag) if ldac_dir else 0
        while remaining > 0:
            cur = burner or model
            n = min(step, remaining)
            if burner is not None:
                n = min(n, burn_mh - burner.sweeps_done)
            if ck_every:
                n = min(n, ck_every - (cur.sweeps_done % ck_every))
            if lag:
                n = min(n, lag - (cur.sweeps_done % lag))
            cur.sweep(n)
            remaining -= n
            mixed = cur.sweeps_done > burnin
            if eval_every > 0 and cur.sweeps_done % eval_every == 0 and mixed:
                ll = cur.record_likelihood()
                if log:
                    log(f"sweep {cur.sweeps_done} loglik {ll:.6e}")
            if ck_every and cur.sweeps_done % ck_every == 0:
                ckpt.save(cur)
            if lag and cur.sweeps_done % lag == 0 and remaining > 0 and mixed:
                from ..io import ldac
                ldac.export_gibbs(ldac_dir, cur, prefix=f"{cur.sweeps_done:03d}")
            if burner is not None and burner.sweeps_done >= burn_mh:
                # hand the chain to the MH model: same documents and tokens, another tiling
                model.load_canonical_z(burner.canonical_z(), burner.sweeps_done, counts_from=burner)
                model.likelihoods = list(burner.likelihoods)
                burner.close()
                burner = dcorpus = None
    model.close()
    if not model.likelihoods or model.likelihoods[-1][0] != model.sweeps_done:
        model.record_likelihood()
    if chains > 1:
        with timer.stage("train"):
            for c in range(1, chains):
                mc = GibbsLDA(corpus, GibbsConfig(K=K, alpha=alpha, beta=beta, seed=(seed + c * 0x9E3779B1) & 0xFFFFFFFF),
                              comm=comm, V_global=int(vocab.numel()))
                mc.plan_average(sweeps)
                mc.initialize()
                mc.sweep(sweeps)
                mc.close()
                # keep only the chain's estimate: its count tables, Δ buffers and posterior sums are
                # freed here instead of living until scoring (HBM grew by (C−1)× a model)
                run.extra_models.append(ChainEstimate(mc.theta(), mc.phi(), mc.sweeps_done))
                del mc
    run.timings.update({"sweeps": sweeps * chains, "chains": chains})
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
    ps = run.pair_scores(run.model.theta(), run.model.phi(), run.pairs.pair_doc, run.pairs.pair_word)
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
    th = run.model.theta()[: run.corpus.D_own]
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
SCORE_SORT_PAIRS = os.environ.get("ONI_SCORE_SORT_PAIRS", "0") == "1"


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
    # the pair-ordered event view costs two 12.5M-element random gathers (inv[order0]) inside the
    # day now that the plan is built per day (0.44 ms), more than the random pair-score reads it
    # saves in k_event_min: off by default here (ONI_SCORE_SORT_PAIRS=1 restores it)
    if SCORE_SORT_PAIRS and ps.order0 is not None:
        plan.order = ps.order0
        plan.inv_sorted = [x[ps.order0].contiguous() for x in invs]
    return plan


@traced("oni:event_score_plan")
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
def plan_score(theta: torch.Tensor, phi: torch.Tensor, plan: ScorePlan, tol: float, hist=None, want_parts=False,
               run: "LdaRun | None" = None):
    """(score, s1, s2) per event in PLAN order (event order unless plan.order is set; map plan
    positions back with plan.order / event indices forward with plan.rank). ``run`` with extra
    chains: pair scores averaged over the chains (:meth:`LdaRun.pair_scores`)."""
    if run is not None and run.extra_models:
        ps = run.pair_scores(theta, phi, plan.pdoc, plan.pword)
    elif plan.tiles is not None:
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
            # same feedback file on every rank: all carry weights, rank 0 adds the tokens
            wts = torch.ones_like(wk, dtype=torch.int32)
            if feedback_here(comm):
                wts = torch.cat([wts, feedback[2].to(torch.int32)])
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
            score, _, _ = plan_score(theta, run.model.phi(), plan, tol, hist=hist, run=run)
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
    if return_pos and comm is not None and comm.dist and comm.world > 1:
        raise ValueError("top_n: positions are only defined on one rank")
    if bmax < 0:
        e = torch.zeros(0, dtype=torch.int64, device=score.device)
        out = (e, torch.zeros(0, dtype=torch.float32, device=score.device))
        return out + (e,) if return_pos else out
    # the local histogram already counts this rank's candidates: no extra pass over the scores
    cap = int(np.cumsum(h_loc)[bmax])
    pos, sc = ops.select_below(score, tol, bmax, cap=max(cap, 1))
    idx = order[pos] if order is not None else pos
    # the ≤ a few thousand candidates come to the host in ONE copy and are ordered there (a chain
    # of tiny device sorts / gathers was ~2 ms of launch and sync gaps per day); results are host
    # tensors
    packed = torch.stack([idx.to(torch.int64), pos.to(torch.int64),
                          sc.view(torch.int32).to(torch.int64)]).cpu().numpy()
    gid = packed[0] + int(row_offset)
    sch = packed[2].astype(np.int32).view(np.float32)
    o = np.lexsort((gid, sch))[:maxresults]  # by score, ties by global row id
    if return_pos:
        return (torch.from_numpy(gid[o].copy()), torch.from_numpy(sch[o].copy()),
                torch.from_numpy(packed[1][o].copy()))
    gid, bits = gid[o], packed[2][o]
    if comm is not None and comm.live:
        # one all-gather of every rank's local top-N (global id, score bits), merged on the host
        loc = torch.from_numpy(np.stack([gid, bits], 1).astype(np.int64)).to(score.device)
        both = torch.cat([p.to(score.device) for p in comm.allgather_var(loc)]).cpu().numpy()
        gid, bits = both[:, 0], both[:, 1]
        o = np.lexsort((gid, bits.astype(np.int32).view(np.float32)))[:maxresults]
        gid, bits = gid[o], bits[o]
    return torch.from_numpy(np.ascontiguousarray(gid)), torch.from_numpy(bits.astype(np.int32).view(np.float32))
