"""Document-term corpus on device: CSR over (doc, word, count) pairs + the SELL token layout.

Replaces the reference's ``reduceByKey((ip, word) -> count)`` + ``zipWithIndex`` dictionaries +
lda-c ``model.dat`` writer (oni-ml OniLDACWrapper.createModel, SURVEY.md §2.2 C20, [U-M]).
Everything here is torch code that runs on the HIP device (sort/unique are rocPRIM radix sorts
inside torch) except the SELL fill, which is a hand-written kernel (csrc/kernels/sell.hip).

Token order inside a document is fixed: pairs sorted by word id, each pair expanded ``count``
times. A token's position in that order (plus the document key) is its RNG identity.
"""
from __future__ import annotations

import math

from dataclasses import dataclass

import torch

from .. import ops
from ..utils.obs import traced

PAD = -1  # 0xFFFFFFFF as int32


@dataclass
class Corpus:
    D: int
    V: int
    T: int
    G: int
    L: int
    doc_keys: torch.Tensor      # int32 [D] (u32 bits): document identity (IP) -> RNG stream
    pair_doc: torch.Tensor      # int32 [nnz]
    pair_word: torch.Tensor     # int32 [nnz]
    pair_cnt: torch.Tensor      # int32 [nnz]
    doc_pair_ptr: torch.Tensor  # int64 [D+1]
    doc_tok_ptr: torch.Tensor   # int64 [D+1]
    pair_tokoff: torch.Tensor   # int64 [nnz] token offset of each pair inside its doc
    slice_off: torch.Tensor     # int64 [ns]
    slice_len: torch.Tensor     # int32 [ns]
    chunk_doc: torch.Tensor     # int32 [ns*S]
    chunk_pos0: torch.Tensor    # int32 [ns*S]
    chunk_len: torch.Tensor     # int32 [ns*S]
    chunk_key: torch.Tensor     # int32 [ns*S]
    chunk_multi: torch.Tensor   # uint8 [ns*S]
    tok_word: torch.Tensor      # int32 [Σ slice_len*S] (PAD = -1)
    long_rows: torch.Tensor     # int32 [n_long] docs split over > 1 chunk
    wsorted: torch.Tensor | None = None  # int32 [T] word ids of all tokens, sorted (recount path)
    wslot: torch.Tensor | None = None    # int32 [T] SELL slot of each word-sorted token
    tile_wlo: torch.Tensor | None = None  # int32 [n_tiles] first word of each recount tile
    tile_whi: torch.Tensor | None = None  # int32 [n_tiles] last word of each recount tile
    wpos: torch.Tensor | None = None      # int32 [SELL slots] word-sorted position of each slot (-1: pad)
    # data parallel with heavy documents cut across ranks (pipeline.common.apply_split): rows
    # [D_own, D) are pieces of split documents; chunk_rng0 is every chunk's GLOBAL canonical
    # position (the Philox counter), chunk_pos0 stays the position inside the local row
    split: dict | None = None
    chunk_rng0: torch.Tensor | None = None

    @property
    def D_own(self) -> int:
        """Rows that are this rank's documents (θ / outputs); the rest are split pieces."""
        return int(self.split["D_own"]) if self.split is not None else self.D

    @property
    def S(self) -> int:
        return 64 // self.G

    @property
    def nnz(self) -> int:
        return int(self.pair_doc.numel())

    @property
    def n_slices(self) -> int:
        return int(self.slice_len.numel())

    @property
    def sell_slots(self) -> int:
        return int(self.tok_word.numel())

    def doc_lengths(self) -> torch.Tensor:
        return self.doc_tok_ptr[1:] - self.doc_tok_ptr[:-1]

    def max_doc_len(self) -> int:
        """Largest doc-topic count a row can hold (a split document's rows hold its global counts)."""
        m = int(self.doc_lengths().max()) if self.D else 0
        return max(m, int(self.split["max_count"])) if self.split is not None else m

    def stats(self) -> dict:
        return {"D": self.D, "V": self.V, "T": self.T, "nnz": self.nnz, "slices": self.n_slices,
                "sell_slots": self.sell_slots, "sell_fill": (self.T / max(self.sell_slots, 1)),
                "long_docs": int(self.long_rows.numel()), "G": self.G, "L": self.L}


def _excl_cumsum(x: torch.Tensor) -> torch.Tensor:
    out = torch.zeros(x.numel() + 1, dtype=torch.int64, device=x.device)
    if x.numel():
        torch.cumsum(x.to(torch.int64), 0, out=out[1:])
    return out


def auto_chunk_len(T_global: int, G: int, lo: int = 32, hi: int = 128) -> int:
    """Chunk length from the GLOBAL token count (so every GPU count picks the same L and the
    chain stays world-size invariant): aim at ~4096 slices of S = 64/G chunks, power of two in
    [lo, hi]. Measured on MI355X: 25M flow tokens → 128 (best of 32..256); 2M DNS tokens at
    K = 50 → 32 (the wave count, not per-token work, bounds small corpora)."""
    S = 64 // G
    want = max(T_global, 1) / (S * 4096.0)
    L = 1 << int(round(math.log2(max(want, 1.0))))
    return int(min(max(L, lo), hi))


# device builds go through the hand-written K08/K09 kernels (csrc/kernels/corpus.hip); the torch
# build below stays as the CPU path and as the bitwise reference of the native one
NATIVE_DEVICE_BUILD = True


@traced("oni:build_corpus")
def build_corpus(tdoc: torch.Tensor, tword: torch.Tensor, D: int, V: int, doc_keys: torch.Tensor, G: int,
                 L: int = 256, weight: torch.Tensor | None = None, pairs=None, native: bool | None = None) -> Corpus:
    """Build pairs/CSR/SELL from token (doc id, word id[, weight]) arrays (any device).

    On a GPU the native kernels run (``pairs``: an already built :class:`oni355.ops.corpus.PairSet`
    of exactly these tokens); ``native=False`` forces the torch reference build."""
    dev = tdoc.device
    if tdoc.numel() != tword.numel():
        raise ValueError("tdoc/tword length mismatch")
    if L < 1 or L > (1 << 20):
        raise ValueError("chunk length L out of range")
    if dev.type == "cuda" and (NATIVE_DEVICE_BUILD if native is None else native):
        return _build_corpus_native(tdoc, tword, D, V, doc_keys, G, L, weight, pairs)
    S = 64 // G
    key = tdoc.to(torch.int64) * V + tword.to(torch.int64)
    if weight is None:
        skey, _ = torch.sort(key)
        uniq, cnt = torch.unique_consecutive(skey, return_counts=True)
    else:
        skey, order = torch.sort(key, stable=True)
        w = weight.to(torch.int64)[order]
        uniq, inv = torch.unique_consecutive(skey, return_inverse=True)
        cnt = torch.zeros(uniq.numel(), dtype=torch.int64, device=dev).index_add_(0, inv, w)
        keep = cnt > 0
        uniq, cnt = uniq[keep], cnt[keep]
    if cnt.numel() and int(cnt.max()) >= 2**31:
        raise ValueError("pair count overflow")
    pair_doc = (uniq // V).to(torch.int32)
    pair_word = (uniq % V).to(torch.int32)
    cnt64 = cnt.to(torch.int64)
    doc_npairs = torch.bincount(pair_doc.to(torch.int64), minlength=D)
    doc_pair_ptr = _excl_cumsum(doc_npairs)
    doc_ntok = torch.zeros(D, dtype=torch.int64, device=dev).index_add_(0, pair_doc.to(torch.int64), cnt64)
    doc_tok_ptr = _excl_cumsum(doc_ntok)
    T = int(doc_tok_ptr[-1])
    glob_excl = torch.cumsum(cnt64, 0) - cnt64
    pair_tokoff = glob_excl - doc_tok_ptr[pair_doc.to(torch.int64)]

    # ---- chunks (≤ L tokens of one doc) --------------------------------------------------------
    nch = (doc_ntok + L - 1) // L
    n_chunks = int(nch.sum())
    cdoc = torch.repeat_interleave(torch.arange(D, device=dev, dtype=torch.int64), nch)
    first = _excl_cumsum(nch)[:-1]
    cidx = torch.arange(n_chunks, device=dev, dtype=torch.int64) - torch.repeat_interleave(first, nch)
    cpos0 = cidx * L
    clen = torch.minimum(torch.full_like(cpos0, L), doc_ntok[cdoc] - cpos0)
    cmulti = (nch[cdoc] > 1)
    # sort by length, longest first (stable: ties keep doc order) -> similar lengths share a wave
    _, order = torch.sort(clen, descending=True, stable=True)
    cdoc, cpos0, clen, cmulti = cdoc[order], cpos0[order], clen[order], cmulti[order]
    n_pad = (-n_chunks) % S
    ns = (n_chunks + n_pad) // S

    def padded(x, fill, dtype):
        out = torch.full((ns * S,), fill, dtype=dtype, device=dev)
        out[:n_chunks] = x.to(dtype)
        return out

    chunk_doc = padded(cdoc, -1, torch.int32)
    chunk_pos0 = padded(cpos0, 0, torch.int32)
    chunk_len = padded(clen, 0, torch.int32)
    chunk_multi = padded(cmulti, 0, torch.uint8)
    chunk_key = torch.zeros(ns * S, dtype=torch.int32, device=dev)
    if n_chunks:
        chunk_key[:n_chunks] = doc_keys.to(torch.int32)[cdoc]
    slice_len = chunk_len.view(ns, S)[:, 0].contiguous() if ns else torch.zeros(0, dtype=torch.int32, device=dev)
    slice_off = _excl_cumsum(slice_len.to(torch.int64) * S)
    total = int(slice_off[-1])
    slice_off = slice_off[:-1].contiguous()
    tok_word = torch.full((max(total, 1),), PAD, dtype=torch.int32, device=dev)
    if n_chunks:
        ops.sell_fill(chunk_doc, chunk_pos0, chunk_len, S, slice_off, doc_pair_ptr, pair_tokoff.contiguous(),
                      pair_word, cnt.to(torch.int32), tok_word)
    long_rows = torch.nonzero(nch > 1).flatten().to(torch.int32)
    # word-sorted token index for the atomic-free n_wk recount (K11 option B)
    slots = torch.nonzero(tok_word != PAD).flatten()
    if slots.numel() >= 2**31:
        raise ValueError("SELL slot index overflows int32")
    wsorted, worder = torch.sort(tok_word[slots], stable=True)
    wslot = slots[worder].to(torch.int32)
    tile = ops.RECOUNT_TILE
    starts = torch.arange(0, wsorted.numel(), tile, device=dev)
    tile_wlo = wsorted[starts].to(torch.int32) if starts.numel() else torch.zeros(0, dtype=torch.int32, device=dev)
    ends = torch.clamp(starts + tile - 1, max=max(wsorted.numel() - 1, 0))
    tile_whi = wsorted[ends].to(torch.int32) if starts.numel() else torch.zeros(0, dtype=torch.int32, device=dev)
    wpos = torch.full((tok_word.numel(),), -1, dtype=torch.int32, device=dev)
    wpos[wslot.long()] = torch.arange(wslot.numel(), dtype=torch.int32, device=dev)
    return Corpus(D=D, V=V, T=T, G=G, L=L, doc_keys=doc_keys.to(torch.int32), pair_doc=pair_doc,
                  pair_word=pair_word, pair_cnt=cnt.to(torch.int32), doc_pair_ptr=doc_pair_ptr,
                  doc_tok_ptr=doc_tok_ptr, pair_tokoff=pair_tokoff.contiguous(), slice_off=slice_off,
                  slice_len=slice_len, chunk_doc=chunk_doc, chunk_pos0=chunk_pos0, chunk_len=chunk_len,
                  chunk_key=chunk_key, chunk_multi=chunk_multi, tok_word=tok_word, long_rows=long_rows,
                  wsorted=wsorted.contiguous(), wslot=wslot.contiguous(), tile_wlo=tile_wlo.contiguous(),
                  tile_whi=tile_whi.contiguous(), wpos=wpos)


def _build_corpus_native(tdoc, tword, D, V, doc_keys, G, L, weight, pairs) -> Corpus:
    from ..ops import corpus as oc
    if weight is not None and bool((weight < 1).any()):
        raise ValueError("token weights must be >= 1 (DUPFACTOR >= 1)")
    if pairs is None:
        pairs = oc.pair_build(tdoc.to(torch.int32).contiguous(), tword.to(torch.int32).contiguous(), D, V,
                              weight.to(torch.int32).contiguous() if weight is not None else None)
    lay = oc.corpus_layout(pairs, doc_keys, G, L, ops.RECOUNT_TILE)
    T = lay.pop("T")
    return Corpus(D=D, V=V, T=T, G=G, L=L, doc_keys=doc_keys.to(torch.int32), pair_doc=pairs.pair_doc,
                  pair_word=pairs.pair_word, pair_cnt=pairs.pair_cnt, **lay)


def canonical_tokens(c: Corpus) -> tuple[torch.Tensor, torch.Tensor]:
    """(doc id, word id) of every token in canonical order (doc-major, word-sorted)."""
    cnt = c.pair_cnt.to(torch.int64)
    return (torch.repeat_interleave(c.pair_doc.to(torch.int64), cnt),
            torch.repeat_interleave(c.pair_word.to(torch.int64), cnt))
