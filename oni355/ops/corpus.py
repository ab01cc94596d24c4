"""K08 / K09 device ops: dictionary encoding, (doc, word) pair build and the SELL corpus layout
(csrc/kernels/corpus.hip). Device tensors only -- the CPU path keeps the torch reference build in
:mod:`oni355.models.corpus`, which these kernels reproduce bit for bit.

Host synchronisation: one 8-byte read per dictionary, one per pair build, one 24-byte read for the
(T, chunks, long docs) totals and one for the SELL slot count -- instead of the dozens of implicit
syncs (``int(tensor)``, ``nonzero``, ``unique``) of the torch build.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib

vp, i64, ci = C.c_void_p, C.c_int64, C.c_int
_SZ = C.POINTER(C.c_size_t)
_lib.register_optional("oni_dict_encode", [vp, i64, ci, vp, vp, vp, vp, vp, vp, _SZ, vp])
_lib.register_optional("oni_hashdict_build", [vp, i64, i64, vp, vp, vp, vp, vp])
_lib.register_optional("oni_hashdict_finish", [vp, i64, ci, i64, vp, vp, vp, i64, vp, vp, vp, _SZ, vp])
_lib.register_optional("oni_route_pack", [vp, vp, vp, vp, vp, i64, ci, vp, vp, vp, vp, _SZ, vp])
_lib.register_optional("oni_route_pack_ids", [vp, vp, vp, vp, vp, i64, ci, vp, vp, vp, vp, _SZ, vp])
_lib.register_optional("oni_route_unpack", [vp, i64, ci, vp, vp, ci, vp, vp, vp, vp, vp])
_lib.register_optional("oni_partition", [vp, vp, vp, i64, ci, vp, vp, vp, vp, vp, _SZ, vp])
_lib.register_optional("oni_place_stats", [vp, vp, i64, vp, i64, ci, vp, vp])
_lib.register_optional("oni_place_owner", [vp, i64, vp, i64, vp, ci, vp, vp, vp])
_lib.register_optional("oni_pair_build", [vp, vp, vp, i64, i64, i64, vp, vp, vp, vp, vp, vp, i64, vp, _SZ, vp])
_lib.register_optional("oni_doc_layout", [vp, vp, i64, i64, ci, vp, vp, vp, vp, vp, vp, vp, _SZ, vp])
_lib.register_optional("oni_chunk_layout", [vp, vp, vp, i64, i64, ci, ci, vp, vp, vp, vp, vp, vp, vp, vp, _SZ, vp])
_lib.register_optional("oni_word_index", [vp, i64, i64, i64, ci, vp, vp, vp, vp, vp, vp, _SZ, vp])


def _call(name: str, *args) -> None:
    """Two-phase launcher: size query (tmp = NULL), scratch from torch's caching allocator, run."""
    L = _lib.lib()
    fn = getattr(L, name)
    nb = C.c_size_t(0)
    _lib.check(fn(*args, None, C.byref(nb), _lib.stream()), name + " (size)")
    tmp = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device="cuda")
    # every launch is on torch's current stream, so the caching allocator may hand this block out
    # again once it is freed here: any later user is stream-ordered behind these kernels
    _lib.check(fn(*args, tmp.data_ptr(), C.byref(nb), _lib.stream()), name)


def _p(t):
    return _lib.ptr(t)


HASH_DICT = True  # tests flip this to compare the two dictionary paths


def bits_for(maxv: int) -> int:
    return max(int(maxv).bit_length(), 1)


HASH_DICT_MIN_KEYS = 1 << 20   # below this the sort path is as fast
HASH_DICT_SLOTS = 1 << 22      # open-addressing table (48 MB): up to 2M distinct keys


def dict_encode_hash(keys64: torch.Tensor, key_bits: int, table_slots: int = HASH_DICT_SLOTS):
    """Hash-table dictionary (csrc/kernels/hashdict.hip): identical output to the sort path, or
    None when the keys have too many distinct values for the table."""
    n = keys64.numel()
    dev = keys64.device
    M = int(table_slots)
    tab = torch.empty(M, dtype=torch.int64, device=dev)
    val = torch.empty(M, dtype=torch.int32, device=dev)
    uns = torch.empty(M // 2 + 1, dtype=torch.int64, device=dev)
    status = torch.zeros(3, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().oni_hashdict_build(_p(keys64), n, M, _p(tab), _p(val), _p(uns), _p(status), _lib.stream()),
               "oni_hashdict_build")
    nu, ovf, _ = (int(x) for x in status.tolist())
    if ovf or nu > M // 2:
        return None
    uniq = torch.empty(max(nu, 1), dtype=torch.int64, device=dev)
    ids = torch.empty(n, dtype=torch.int32, device=dev)
    _call("oni_hashdict_finish", _p(keys64), n, int(min(max(key_bits, 1), 64)), M, _p(tab), _p(val), _p(uns), nu,
          _p(uniq), _p(ids))
    return uniq[:nu], ids


def dict_encode(keys64: torch.Tensor, key_bits: int = 64, weights: torch.Tensor | None = None,
                counts: bool = False, hashed: bool = False):
    """Sorted unique keys (int64) and the int32 id of every key (``torch.unique(return_inverse)``).

    ``counts=True`` also returns Σ weights (int64; 1 per key without ``weights``) of every unique
    key, read off the sorted runs (``torch.unique(return_counts)`` with weights). ``hashed``: large
    inputs of keys below 2^63 try the hash-table path (:func:`dict_encode_hash`) first -- a win for
    few distinct keys (the word vocabulary: 2.06 -> 1.01 ms at 25M keys / 5.7k words), a loss for
    many (IP documents: 370k distinct, the sort path stays 1.6 ms faster)."""
    if keys64.dtype != torch.int64 or not keys64.is_contiguous():
        raise TypeError("dict_encode: contiguous int64 keys")
    n = keys64.numel()
    if hashed and not counts and n >= HASH_DICT_MIN_KEYS and key_bits <= 62 and HASH_DICT:
        r = dict_encode_hash(keys64, key_bits)
        if r is not None:
            return r
    if weights is not None and (weights.dtype != torch.int32 or weights.numel() != n):
        raise TypeError("dict_encode: weights must be int32 [n]")
    dev = keys64.device
    uniq = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    ids = torch.empty(n, dtype=torch.int32, device=dev)
    nu = torch.zeros(1, dtype=torch.int64, device=dev)
    cnt = torch.empty(max(n, 1), dtype=torch.int64, device=dev) if counts else None
    _call("oni_dict_encode", _p(keys64), n, int(min(max(key_bits, 1), 64)), _p(uniq), _p(ids) if n else None, _p(nu),
          _p(weights.contiguous()) if weights is not None else None, _p(cnt) if counts else None)
    u = int(nu.item())
    return (uniq[:u], ids, cnt[:u]) if counts else (uniq[:u], ids)


def route_pack(owner_of_id: torch.Tensor, ids: torch.Tensor, keys64: torch.Tensor, word: torch.Tensor,
               weight: torch.Tensor | None, world: int):
    """All-to-all send buffer of the token routing (csrc/kernels/route.hip): (send int32 [n, 2|3]
    grouped by owner rank, order int32 [n] = token of each slot, counts int64 [world])."""
    n = ids.numel()
    for t, nm, dt in ((owner_of_id, "owner_of_id", torch.int32), (ids, "ids", torch.int32),
                      (keys64, "keys64", torch.int64), (word, "word", torch.int32)):
        if t.dtype != dt or not t.is_contiguous():
            raise TypeError(f"route_pack: {nm} must be contiguous {dt}")
    if keys64.numel() != n or word.numel() != n or (weight is not None and weight.numel() != n):
        raise ValueError("route_pack: token arrays differ in length")
    if not 1 <= world <= 256:
        raise ValueError("route_pack: 1 <= world <= 256")
    dev = ids.device
    C = 3 if weight is not None else 2
    send = torch.empty((n, C), dtype=torch.int32, device=dev)
    order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    _call("oni_route_pack", _p(owner_of_id), _p(ids), _p(keys64), _p(word),
          _p(weight.to(torch.int32).contiguous()) if weight is not None else None, n, int(world), _p(send),
          _p(order), _p(counts))
    return send, order[:n], counts


def route_pack_ids(owner_of_id: torch.Tensor, ids: torch.Tensor, doc_val: torch.Tensor, word: torch.Tensor,
                   weight: torch.Tensor | None, world: int):
    """:func:`route_pack` whose column 0 carries ``doc_val[ids[t]]`` (int32 per local document:
    its index in the key list sent to the owner) instead of the token's doc key."""
    n = ids.numel()
    for t, nm in ((owner_of_id, "owner_of_id"), (ids, "ids"), (doc_val, "doc_val"), (word, "word")):
        if t.dtype != torch.int32 or not t.is_contiguous():
            raise TypeError(f"route_pack_ids: {nm} must be contiguous int32")
    if doc_val.numel() != owner_of_id.numel():
        raise ValueError("route_pack_ids: doc_val and owner_of_id cover different documents")
    if word.numel() != n or (weight is not None and weight.numel() != n):
        raise ValueError("route_pack_ids: token arrays differ in length")
    if not 1 <= world <= 256:
        raise ValueError("route_pack_ids: 1 <= world <= 256")
    dev = ids.device
    C = 3 if weight is not None else 2
    send = torch.empty((n, C), dtype=torch.int32, device=dev)
    order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    _call("oni_route_pack_ids", _p(owner_of_id), _p(ids), _p(doc_val), _p(word),
          _p(weight.to(torch.int32).contiguous()) if weight is not None else None, n, int(world), _p(send),
          _p(order), _p(counts))
    return send, order[:n], counts


def partition(owner_of_id: torch.Tensor, world: int, ids: torch.Tensor | None = None,
              keys64: torch.Tensor | None = None, rank: bool = False):
    """Stable partition of items by owner rank (csrc/kernels/route.hip ``oni_partition``): item i's
    owner is ``owner_of_id[ids[i]]`` (``owner_of_id[i]`` without ``ids``). Returns (order int32 [n]
    = item of each slot, counts int64 [world], rank int32 [n] = slot of each item within its
    owner's group or None, u32 bits of ``keys64`` at each slot int32 [n] or None) -- a stable
    ``argsort(owner)`` with the group offsets and a gather, in two passes over the items."""
    if owner_of_id.dtype != torch.int32 or not owner_of_id.is_contiguous():
        raise TypeError("partition: owner_of_id must be contiguous int32")
    if ids is not None and (ids.dtype != torch.int32 or not ids.is_contiguous()):
        raise TypeError("partition: ids must be contiguous int32")
    n = ids.numel() if ids is not None else owner_of_id.numel()
    if keys64 is not None and (keys64.dtype != torch.int64 or not keys64.is_contiguous() or keys64.numel() != n):
        raise TypeError("partition: keys64 must be contiguous int64 [n]")
    if not 1 <= world <= 256:
        raise ValueError("partition: 1 <= world <= 256")
    dev = owner_of_id.device
    order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    rk = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if rank else None
    ko = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if keys64 is not None else None
    _call("oni_partition", _p(owner_of_id), _p(ids) if ids is not None else None,
          _p(keys64) if keys64 is not None else None, n, int(world), _p(order), _p(rk) if rank else None,
          _p(ko) if ko is not None else None, _p(counts))
    return order[:n], counts, (rk[:n] if rank else None), (ko[:n] if ko is not None else None)


def place_stats(ukeys: torch.Tensor, ucnt: torch.Tensor, cand: torch.Tensor, B: int) -> torch.Tensor:
    """int64 [nc + B]: the local count of every candidate document (0 when absent here), then the
    summed counts of the other documents per hash bucket (``pipeline.common.doc_owner(key, B)``).
    ``ukeys`` and ``cand`` ascending int64."""
    for t, nm in ((ukeys, "ukeys"), (ucnt, "ucnt"), (cand, "cand")):
        if t.dtype != torch.int64 or not t.is_contiguous():
            raise TypeError(f"place_stats: {nm} must be contiguous int64")
    if ucnt.numel() != ukeys.numel() or B < 1:
        raise ValueError("place_stats: one count per key, B >= 1")
    both = torch.empty(cand.numel() + B, dtype=torch.int64, device=ukeys.device)
    _lib.check(_lib.lib().oni_place_stats(_p(ukeys), _p(ucnt), ukeys.numel(), _p(cand), cand.numel(), int(B), _p(both),
                                          _lib.stream()), "oni_place_stats")
    return both


def place_owner(ukeys: torch.Tensor, cand: torch.Tensor, cown: torch.Tensor, bown: torch.Tensor) -> torch.Tensor:
    """int32 owner of every document: ``cown[j]`` for the candidate ``cand[j]``, else the owner
    ``bown`` of its hash bucket."""
    if ukeys.dtype != torch.int64 or cand.dtype != torch.int64 or not (ukeys.is_contiguous() and cand.is_contiguous()):
        raise TypeError("place_owner: contiguous int64 keys")
    if cown.dtype != torch.int32 or bown.dtype != torch.int32 or cown.numel() != cand.numel() or bown.numel() < 1:
        raise TypeError("place_owner: int32 owners, one per candidate, >= 1 bucket")
    uown = torch.empty(ukeys.numel(), dtype=torch.int32, device=ukeys.device)
    _lib.check(_lib.lib().oni_place_owner(_p(ukeys), ukeys.numel(), _p(cand), cand.numel(), _p(cown.contiguous()),
                                          int(bown.numel()), _p(bown.contiguous()), _p(uown), _lib.stream()),
               "oni_place_owner")
    return uown


def route_unpack(recv: torch.Tensor, recv_counts: list, key_counts: list, kid: torch.Tensor, weights: bool):
    """Owner side of :func:`route_pack_ids`: ``recv`` [n, C] int32 rows grouped by source rank
    (``recv_counts`` rows each), column 0 an index into that source's key list (``key_counts``
    entries each, concatenated in rank order; ``kid`` = dictionary id of every entry). Returns
    (doc id, word id, weight) int32 [n] (weight all ones without ``weights``)."""
    W = len(recv_counts)
    if len(key_counts) != W or not 1 <= W <= 256:
        raise ValueError("route_unpack: one count per source rank, 1 <= world <= 256")
    if recv.dtype != torch.int32 or recv.dim() != 2 or not recv.is_contiguous():
        raise TypeError("route_unpack: recv must be contiguous int32 [n, C]")
    n, C = int(recv.shape[0]), int(recv.shape[1])
    if n != sum(int(x) for x in recv_counts) or kid.numel() < sum(int(x) for x in key_counts):
        raise ValueError("route_unpack: counts do not match the buffers")
    if kid.dtype != torch.int32 or not kid.is_contiguous():
        raise TypeError("route_unpack: kid must be contiguous int32")
    dev = recv.device
    seg = [0]
    for x in recv_counts:
        seg.append(seg[-1] + int(x))
    koff = [0]
    for x in key_counts[:-1]:
        koff.append(koff[-1] + int(x))
    meta = torch.tensor(seg + koff, dtype=torch.int64).to(dev, non_blocking=True)
    doc = torch.empty(n, dtype=torch.int32, device=dev)
    word = torch.empty(n, dtype=torch.int32, device=dev)
    wt = torch.empty(n, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().oni_route_unpack(_p(recv), n, C, _p(meta), _lib.ptr(meta) + 8 * (W + 1), W, _p(kid),
                                           _p(doc), _p(word), _p(wt), _lib.stream()), "oni_route_unpack")
    return doc, word, wt


@dataclass
class PairSet:
    """Distinct (doc, word) pairs of a token list (doc-major, word-sorted) + per-token pair index."""
    pair_doc: torch.Tensor   # int32 [nnz]
    pair_word: torch.Tensor  # int32 [nnz]
    pair_cnt: torch.Tensor   # int32 [nnz] Σ weights
    tok_pair: torch.Tensor   # int32 [n] pair of every token
    order0: torch.Tensor | None  # int64 [n0] tokens < n0 in (pair, position) order
    D: int
    V: int

    @property
    def nnz(self) -> int:
        return int(self.pair_doc.numel())


def pair_build(doc: torch.Tensor, word: torch.Tensor, D: int, V: int, weight: torch.Tensor | None = None,
               n0: int = 0) -> PairSet:
    n = doc.numel()
    for t, nm in ((doc, "doc"), (word, "word")):
        if t.dtype != torch.int32 or not t.is_contiguous() or t.numel() != n:
            raise TypeError(f"pair_build: {nm} must be contiguous int32 [{n}]")
    if weight is not None and (weight.dtype != torch.int32 or weight.numel() != n):
        raise TypeError("pair_build: weight must be int32 [n]")
    if not 0 <= n0 <= n:
        raise ValueError("pair_build: n0 out of range")
    dev = doc.device
    pd = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    pw = torch.empty_like(pd)
    pc = torch.empty_like(pd)
    tp = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    nnz = torch.zeros(1, dtype=torch.int64, device=dev)
    o0 = torch.empty(max(n0, 1), dtype=torch.int32, device=dev) if n0 > 0 else None
    _call("oni_pair_build", _p(doc), _p(word), _p(weight.contiguous()) if weight is not None else None, n, int(D), int(V),
          _p(pd), _p(pw), _p(pc), _p(tp), _p(nnz), _p(o0) if o0 is not None else None, int(n0))
    m = int(nnz.item())
    return PairSet(pd[:m], pw[:m], pc[:m], tp[:n], o0.to(torch.int64) if o0 is not None else None, int(D), int(V))


def corpus_layout(ps: PairSet, doc_keys: torch.Tensor, G: int, L: int, recount_tile: int):
    """CSR + chunk + SELL + word-index tables of :class:`oni355.models.corpus.Corpus` from pairs."""
    from .. import ops
    dev = ps.pair_doc.device
    D, V, nnz = ps.D, ps.V, ps.nnz
    S = 64 // G
    i64t, i32t = torch.int64, torch.int32
    doc_pair_ptr = torch.empty(D + 1, dtype=i64t, device=dev)
    doc_tok_ptr = torch.empty(D + 1, dtype=i64t, device=dev)
    pair_tokoff = torch.empty(max(nnz, 1), dtype=i64t, device=dev)
    chunk_first = torch.empty(D + 1, dtype=i64t, device=dev)
    long_rows = torch.empty(max(D, 1), dtype=i32t, device=dev)
    scal = torch.zeros(3, dtype=i64t, device=dev)
    _call("oni_doc_layout", _p(ps.pair_doc) if nnz else None, _p(ps.pair_cnt) if nnz else None, nnz, D, int(L),
          _p(doc_pair_ptr), _p(doc_tok_ptr), _p(pair_tokoff), _p(chunk_first), _p(long_rows), _p(scal))
    T, n_chunks, n_long = (int(x) for x in scal.tolist())
    ns = (n_chunks + S - 1) // S
    dk = doc_keys.to(i32t).contiguous()
    chunk_doc = torch.empty(max(ns * S, 1), dtype=i32t, device=dev)
    chunk_pos0 = torch.empty_like(chunk_doc)
    chunk_len = torch.empty_like(chunk_doc)
    chunk_multi = torch.empty(max(ns * S, 1), dtype=torch.uint8, device=dev)
    chunk_key = torch.empty_like(chunk_doc)
    slice_len = torch.empty(max(ns, 1), dtype=i32t, device=dev)
    slice_off = torch.empty(ns + 1, dtype=i64t, device=dev)
    _call("oni_chunk_layout", _p(chunk_first), _p(doc_tok_ptr), _p(dk) if D else None, D, n_chunks, int(L), S,
          _p(chunk_doc), _p(chunk_pos0), _p(chunk_len), _p(chunk_multi), _p(chunk_key), _p(slice_len),
          _p(slice_off))
    total = int(slice_off[-1].item())
    chunk_doc, chunk_pos0, chunk_len = chunk_doc[: ns * S], chunk_pos0[: ns * S], chunk_len[: ns * S]
    chunk_multi, chunk_key, slice_len = chunk_multi[: ns * S], chunk_key[: ns * S], slice_len[:ns]
    tok_word = torch.full((max(total, 1),), -1, dtype=i32t, device=dev)
    if n_chunks:
        ops.sell_fill(chunk_doc, chunk_pos0, chunk_len, S, slice_off[:ns].contiguous(), doc_pair_ptr,
                      pair_tokoff[:nnz].contiguous(), ps.pair_word, ps.pair_cnt, tok_word)
    slots = tok_word.numel()
    n_tiles = (T + recount_tile - 1) // recount_tile
    wsorted = torch.empty(max(slots, 1), dtype=i32t, device=dev)  # sorted in place; [:T] are the tokens
    wslot = torch.empty_like(wsorted)
    wpos = torch.empty(slots, dtype=i32t, device=dev)
    tile_wlo = torch.empty(max(n_tiles, 1), dtype=i32t, device=dev)
    tile_whi = torch.empty_like(tile_wlo)
    _call("oni_word_index", _p(tok_word), slots, T, V, int(recount_tile), _p(wsorted), _p(wslot), _p(wpos),
          _p(tile_wlo), _p(tile_whi))
    return dict(T=T, doc_pair_ptr=doc_pair_ptr, doc_tok_ptr=doc_tok_ptr, pair_tokoff=pair_tokoff[:nnz],
                slice_off=slice_off[:ns].contiguous(), slice_len=slice_len, chunk_doc=chunk_doc,
                chunk_pos0=chunk_pos0, chunk_len=chunk_len, chunk_key=chunk_key, chunk_multi=chunk_multi,
                tok_word=tok_word, long_rows=long_rows[:n_long], wsorted=wsorted[:T], wslot=wslot[:T],
                tile_wlo=tile_wlo[:n_tiles], tile_whi=tile_whi[:n_tiles], wpos=wpos)
