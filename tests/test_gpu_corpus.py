"""Native K08/K09 (csrc/kernels/corpus.hip) == the torch reference build, field by field, at awkward
and bench-like sizes; dictionary encode == torch.unique; pair-derived score plans == score_plan."""
import numpy as np
import pytest
import torch

from oni355.models.corpus import build_corpus
from oni355.ops import corpus as oc
from oni355.pipeline import common

pytestmark = pytest.mark.gpu

FIELDS = ("pair_doc", "pair_word", "pair_cnt", "doc_pair_ptr", "doc_tok_ptr", "pair_tokoff", "slice_off",
          "slice_len", "chunk_doc", "chunk_pos0", "chunk_len", "chunk_key", "chunk_multi", "tok_word", "long_rows",
          "wsorted", "wslot", "tile_wlo", "tile_whi", "wpos", "doc_keys")


def _tokens(n, D, V, seed, zipf=True):
    r = np.random.default_rng(seed)
    if zipf:
        p = 1.0 / np.arange(1, D + 1) ** 1.1
        doc = r.choice(D, n, p=p / p.sum())
    else:
        doc = r.integers(0, D, n)
    word = np.minimum(r.zipf(1.3, n) - 1, V - 1)
    doc[:D] = np.arange(D)  # every doc id present (dense ids, as after dictionary encoding)
    return torch.from_numpy(doc.astype(np.int64)), torch.from_numpy(word.astype(np.int64))


@pytest.mark.parametrize("n,D,V,G,L,weighted", [(1, 1, 1, 1, 32, False), (65, 63, 64, 1, 32, False),
                                                (5000, 300, 200, 1, 64, True), (20000, 700, 900, 4, 128, False),
                                                (200_003, 4000, 3000, 8, 128, True), (2_500_000, 60_000, 6000, 1, 128, False)])
def test_native_corpus_equals_torch_build(gpu, n, D, V, G, L, weighted):
    tdoc, tword = _tokens(n, D, V, seed=n)
    keys = (torch.arange(D, dtype=torch.int64) * 2654435761 & 0xFFFFFFFF).to(torch.int64)
    keys32 = common.i64_to_u32bits(keys)
    w = None
    if weighted:
        w = torch.ones(n, dtype=torch.int64)
        w[::97] = 1000
    ref = build_corpus(tdoc.to(gpu), tword.to(gpu), D, V, keys32.to(gpu), G, L=L,
                       weight=None if w is None else w.to(gpu), native=False)
    nat = build_corpus(tdoc.to(gpu), tword.to(gpu), D, V, keys32.to(gpu), G, L=L,
                       weight=None if w is None else w.to(gpu), native=True)
    assert nat.T == ref.T and nat.D == ref.D
    for f in FIELDS:
        a, b = getattr(ref, f), getattr(nat, f)
        assert a.dtype == b.dtype, f
        assert torch.equal(a.cpu(), b.cpu()), f


@pytest.mark.parametrize("n,bits", [(1, 32), (1000, 32), (3_000_001, 32), (100_000, 40), (2_200_000, 40), (77, 64)])
def test_dict_encode_equals_unique(gpu, n, bits):
    r = np.random.default_rng(n)
    table = r.integers(0, 2 ** min(bits, 62), max(n // 3, 1), dtype=np.int64)
    keys = torch.from_numpy(table[r.integers(0, table.size, n)])
    u, inv = torch.unique(keys, return_inverse=True)
    nu, ni = oc.dict_encode(keys.to(gpu).contiguous(), bits)
    assert torch.equal(u, nu.cpu()) and torch.equal(inv.to(torch.int32), ni.cpu())


def test_pair_plan_equals_score_plan(gpu, monkeypatch):
    r = np.random.default_rng(5)
    n, D, V = 50_000, 900, 700
    dkeys = torch.from_numpy(np.sort(r.choice(2**32, D, replace=False)).astype(np.int64))
    vocab = torch.from_numpy(np.sort(r.choice(2**29, V, replace=False)).astype(np.int64))
    sides = [(dkeys[torch.from_numpy(r.integers(0, D, n))], vocab[torch.from_numpy(r.integers(0, V, n))])
             for _ in range(2)]
    g = [(a.to(gpu), b.to(gpu)) for a, b in sides]
    ref = common.score_plan(dkeys.to(gpu), vocab.to(gpu), g, tiles=False, sort_events=True)
    doc_all = torch.cat([a for a, _ in g])
    ud, dids = common.encode_docs(doc_all)
    wids = torch.searchsorted(vocab.to(gpu), torch.cat([b for _, b in g])).to(torch.int32)
    ps = oc.pair_build(dids, wids.contiguous(), int(ud.numel()), V, n0=n)
    plan = common.plan_from_pairs(ps, n, 2, doc_rows=common.lookup(dkeys.to(gpu), ud))
    assert torch.equal(ref.pdoc, plan.pdoc) and torch.equal(ref.pword, plan.pword)
    for a, b in zip(ref.inv, plan.inv):
        assert torch.equal(a, b)
    assert plan.order is None  # the per-day plan scores events in event order by default
    # the pair-ordered event view (ONI_SCORE_SORT_PAIRS=1) equals score_plan's
    monkeypatch.setattr(common, "SCORE_SORT_PAIRS", True)
    plan = common.plan_from_pairs(ps, n, 2, doc_rows=common.lookup(dkeys.to(gpu), ud))
    assert torch.equal(ref.order, plan.order) and torch.equal(ref.rank, plan.rank)


def test_flow_pipeline_native_equals_torch_corpus(gpu, monkeypatch):
    """End to end: the run with the native corpus/score plan == the run with the torch builds."""
    from oni355.models import corpus as cm
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    day = generate_flows(30_000, seed=8)
    a = run_flow(day.cols, K=20, sweeps=6, maxresults=300, device="cuda:0")
    monkeypatch.setattr(cm, "NATIVE_DEVICE_BUILD", False)
    b = run_flow(day.cols, K=20, sweeps=6, maxresults=300, device="cuda:0")
    assert np.array_equal(a.rows, b.rows) and np.array_equal(a.scores, b.scores)
    assert a.stats["loglik"] == b.stats["loglik"]


@pytest.mark.parametrize("n,weighted", [(1, False), (5000, True), (2_200_000, False), (1_000_003, True)])
def test_dict_encode_counts_equal_weighted_unique(gpu, n, weighted):
    """Per-key token counts (the DP placement's document loads) == torch.unique counts / index_add."""
    r = np.random.default_rng(n + 7)
    keys = torch.from_numpy((r.zipf(1.2, n) * 2654435761 % 2**32).astype(np.int64))
    w = torch.from_numpy(r.integers(1, 1000, n).astype(np.int32)) if weighted else None
    u, inv = torch.unique(keys, return_inverse=True)
    ref = torch.zeros(u.numel(), dtype=torch.int64).index_add_(0, inv, w.to(torch.int64) if weighted else
                                                              torch.ones(n, dtype=torch.int64))
    nu, ni, nc = oc.dict_encode(keys.to(gpu).contiguous(), 32, w.to(gpu) if weighted else None, counts=True)
    assert torch.equal(u, nu.cpu()) and torch.equal(inv.to(torch.int32), ni.cpu())
    assert torch.equal(ref, nc.cpu())


@pytest.mark.parametrize("n,W,weighted", [(1, 1, False), (1000, 2, True), (777_777, 3, False), (2_000_000, 8, True)])
def test_route_pack_is_stable_owner_partition(gpu, n, W, weighted):
    """route_pack == stable argsort by owner + gathered (doc key, word[, weight]) columns + counts."""
    r = np.random.default_rng(n)
    U = max(n // 5, 1)
    ids = torch.from_numpy(r.integers(0, U, n).astype(np.int32))
    own = torch.from_numpy(r.integers(0, W, U).astype(np.int32))
    keys = torch.from_numpy(r.integers(0, 2**32, n, dtype=np.int64))
    word = torch.from_numpy(r.integers(0, 10**6, n).astype(np.int32))
    wt = torch.from_numpy(r.integers(1, 5, n).astype(np.int32)) if weighted else None
    send, order, counts = oc.route_pack(own.to(gpu), ids.to(gpu), keys.to(gpu), word.to(gpu),
                                        wt.to(gpu) if weighted else None, W)
    tok_own = own[ids.long()].long()
    ref_order = torch.argsort(tok_own, stable=True)
    assert torch.equal(order.cpu().long(), ref_order)
    assert torch.equal(counts.cpu(), torch.bincount(tok_own, minlength=W))
    cols = [common.i64_to_u32bits(keys[ref_order]), word[ref_order]] + ([wt[ref_order]] if weighted else [])
    assert torch.equal(send.cpu(), torch.stack(cols, 1))


@pytest.mark.parametrize("n,W", [(0, 1), (1, 1), (5000, 2), (2049, 64), (1_234_567, 8), (300_000, 256)])
def test_partition_is_stable_argsort_with_ranks(gpu, n, W):
    """oni_partition == stable argsort by owner (order), bincount (counts), slot within the owner
    group (rank) and the keys' u32 bits in slot order -- with and without an id indirection."""
    r = np.random.default_rng(n + W)
    U = max(n // 3, 1)
    own = torch.from_numpy(r.integers(0, W, U).astype(np.int32))
    ids = torch.from_numpy(r.integers(0, U, n).astype(np.int32))
    keys = torch.from_numpy(r.integers(0, 2**32, n, dtype=np.int64))
    order, counts, rank, kout = oc.partition(own.to(gpu), W, ids=ids.to(gpu), keys64=keys.to(gpu), rank=True)
    tok = own[ids.long()].long()
    ref = torch.argsort(tok, stable=True)
    assert torch.equal(order.cpu().long(), ref)
    cnt = torch.bincount(tok, minlength=W)
    assert torch.equal(counts.cpu(), cnt)
    start = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(cnt, 0)[:-1]])
    ref_rank = torch.empty(n, dtype=torch.int64)
    ref_rank[ref] = torch.arange(n) - start[tok[ref]]
    assert torch.equal(rank.cpu().long(), ref_rank)
    assert torch.equal(kout.cpu(), common.i64_to_u32bits(keys[ref]))
    o2, c2, _, _ = oc.partition(own.to(gpu), W)  # documents themselves
    assert torch.equal(o2.cpu().long(), torch.argsort(own.long(), stable=True))
    assert torch.equal(c2.cpu(), torch.bincount(own.long(), minlength=W))


@pytest.mark.parametrize("U,B,nc", [(1, 1, 0), (10_000, 64, 37), (500_000, 512, 4096), (200_000, 8192, 100)])
def test_place_kernels_match_torch_twins(gpu, U, B, nc):
    """place_stats / place_owner (csrc/kernels/route.hip) == the torch twins place_docs uses on the
    CPU: candidate counts, hash-bucket loads (LDS and global-atomic bucket paths) and owners."""
    r = np.random.default_rng(U + B)
    ukeys = torch.from_numpy(np.unique(r.integers(0, 2**32, U, dtype=np.int64)))
    ucnt = torch.from_numpy(r.zipf(1.3, ukeys.numel()).clip(max=10**6).astype(np.int64))
    extra = torch.from_numpy(r.integers(0, 2**32, nc // 2, dtype=np.int64))  # candidates absent here
    cand = torch.unique(torch.cat([ukeys[torch.from_numpy(r.permutation(ukeys.numel())[: nc - nc // 2])], extra]))
    both = oc.place_stats(ukeys.to(gpu), ucnt.to(gpu), cand.to(gpu), B)
    assert torch.equal(both.cpu(), common._place_stats_ref(ukeys, ucnt, cand, B))
    cown = torch.from_numpy(r.integers(0, 8, cand.numel()).astype(np.int32))
    bown = torch.from_numpy(r.integers(0, 8, B).astype(np.int32))
    got = oc.place_owner(ukeys.to(gpu), cand.to(gpu), cown.to(gpu), bown.to(gpu))
    assert torch.equal(got.cpu(), common._place_owner_ref(ukeys, cand, cown, bown))


@pytest.mark.parametrize("W,weighted", [(1, False), (3, True), (8, False)])
def test_route_ids_unpack_equals_key_routing(gpu, W, weighted):
    """Id routing (route_pack_ids at every source + key lists + route_unpack at the owner) gives
    the owner exactly encode_docs() of the doc keys it would have received, with the same words
    and weights in the same row order. W source ranks are simulated on one device."""
    r = np.random.default_rng(W)
    uni = np.unique(r.integers(0, 2**32, 50_000, dtype=np.int64))
    srcs = []
    for s_ in range(W):
        n = int(r.integers(100_000, 300_000))
        keys = torch.from_numpy(uni[(r.zipf(1.3, n) - 1) % uni.size]).to(gpu)
        word = torch.from_numpy(r.integers(0, 10**5, n).astype(np.int32)).to(gpu)
        wt = torch.from_numpy(r.integers(1, 5, n).astype(np.int32)).to(gpu) if weighted else None
        ukeys, ids = oc.dict_encode(keys, 32)
        own = ((ukeys * 0x9E3779B1 & 0xFFFFFFFF) >> 16) % W
        uown = own.to(torch.int32).contiguous()
        kperm = torch.argsort(uown, stable=True)
        kcnt = torch.bincount(uown.long(), minlength=W)
        kst = torch.cat([torch.zeros(1, dtype=torch.int64, device=gpu), torch.cumsum(kcnt, 0)])
        pos = torch.empty_like(uown)
        pos[kperm] = (torch.arange(ukeys.numel(), device=gpu) - kst[uown[kperm].long()]).to(torch.int32)
        send, order, counts = oc.route_pack_ids(uown, ids, pos, word, wt, W)
        ref_send, ref_order, ref_counts = oc.route_pack(uown, ids, keys, word, wt, W)
        assert torch.equal(order, ref_order) and torch.equal(counts, ref_counts)
        assert torch.equal(send[:, 1:], ref_send[:, 1:])
        srcs.append((send, counts.tolist(), ukeys[kperm], kcnt.tolist(), ref_send))
    for o in range(W):
        rows, rc, klists, krc, ref_rows = [], [], [], [], []
        for send, counts, klist, kcnt, ref_send in srcs:
            a = sum(counts[:o])
            rows.append(send[a:a + counts[o]])
            ref_rows.append(ref_send[a:a + counts[o]])
            rc.append(counts[o])
            b = sum(kcnt[:o])
            klists.append(klist[b:b + kcnt[o]])
            krc.append(kcnt[o])
        recv = torch.cat(rows).contiguous()
        udoc, kid = oc.dict_encode(torch.cat(klists).contiguous(), 32)
        doc, word, wt = oc.route_unpack(recv, rc, krc, kid, weighted)
        ref = torch.cat(ref_rows)
        rdoc_u, rdoc = oc.dict_encode(common.u32_to_i64(ref[:, 0]).contiguous(), 32)
        assert torch.equal(udoc, rdoc_u) and torch.equal(doc, rdoc)
        assert torch.equal(word, ref[:, 1])
        assert torch.equal(wt, ref[:, 2] if weighted else torch.ones_like(word))


@pytest.mark.parametrize("n,distinct,bits", [(1 << 20, 6000, 30), (3_000_001, 400_000, 32), (2_000_000, 3, 8),
                                             (1_500_000, 1_400_000, 40), (25_000_000, 5733, 29)])
def test_hash_dictionary_equals_sort_path(gpu, n, distinct, bits):
    """The hash-table dictionary (hashdict.hip) == the radix-sort dictionary, bitwise, incl. Zipf
    hot keys; a key set too large for the table falls back to the sort path."""
    r = np.random.default_rng(n)
    table = np.unique(r.integers(0, 2 ** bits, distinct * 2, dtype=np.int64))[:distinct]
    p = 1.0 / np.arange(1, table.size + 1) ** 1.1
    keys = torch.from_numpy(table[r.choice(table.size, n, p=p / p.sum())]).to(gpu).contiguous()
    oc.HASH_DICT = False
    try:
        su, si = oc.dict_encode(keys, bits)
    finally:
        oc.HASH_DICT = True
    hu, hi = oc.dict_encode(keys, bits, hashed=True)
    assert torch.equal(su, hu) and torch.equal(si, hi)
    small = oc.dict_encode_hash(keys, bits, table_slots=1 << 10)
    assert (small is None) == (int(su.numel()) > (1 << 9))
