"""Data-parallel correctness without a GPU cluster: gloo, world_size 2 and 3, CPU tensors.

The DP design (owner-routed documents, global vocabulary, sweep-start snapshots, Philox keyed by
(doc, pos)) makes every sample independent of the rank count, so a multi-rank run must reproduce
the single-process run's top-N rows and scores exactly.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, out_q, env=None):
    os.environ.update(env or {})
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    comm = pc.init_from_env("cpu")
    day = generate_flows(n_total, seed=11)
    per = n_total // world
    lo = rank * per
    hi = n_total if rank == world - 1 else lo + per
    cols = {k: v[lo:hi] for k, v in day.cols.items()}
    res = run_flow(cols, K=20, sweeps=4, maxresults=150, device="cpu", comm=comm, row_offset=lo)
    if rank == 0:
        out_q.put((res.rows, res.scores, res.src_scores, res.dst_scores, res.stats["loglik"]))
    comm.barrier()
    pc.shutdown()


def _run_world(world, n_total, env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,env", [(2, None), (3, None), (2, {"ONI_X01_PACK": "1"}),
                                       (3, {"ONI_X01_PACK": "1", "ONI_X01_LIGHT_MAX": "40"}),
                                       (3, {"ONI_X01_PACK": "1", "ONI_X01_LIGHT_MAX": "40", "ONI_X01_TINY_MAX": "6"}),
                                       (2, {"ONI_X01_PACK": "auto", "ONI_X01_PACK_MIN_BYTES": "0"})])
def test_dp_matches_single_process(world, env):
    """Also with the packed X01 payload forced into a light/heavy word mix, and unpacked."""
    n = 6000
    one = _run_world(1, n)
    many = _run_world(world, n, env)
    assert np.array_equal(one[0], many[0])
    assert np.array_equal(one[1], many[1])
    assert np.array_equal(one[2], many[2]) and np.array_equal(one[3], many[3])
    assert one[4] == pytest.approx(many[4], rel=1e-9)


def test_balanced_owner_evens_out_power_law_docs():
    import numpy as np
    import torch

    from oni355.pipeline import common

    class _Comm:
        world = 8
        dist = live = True

        def allgather_var(self, t):
            return [t]

        def allreduce_(self, t):
            return t

    r = np.random.default_rng(0)
    keys = torch.from_numpy(r.zipf(1.1, 400_000).astype(np.int64) * 7919 % (2**32))  # top doc ~9 % < 1/8
    w = torch.ones_like(keys)
    own = common.balanced_owner(keys, w, _Comm())
    load = torch.bincount(own, minlength=8).double()
    hashed = torch.bincount(common.doc_owner(keys, 8), minlength=8).double()
    assert float(load.max() / load.mean()) < 1.05 < float(hashed.max() / hashed.mean())
    # same doc -> same owner
    u, inv = torch.unique(keys, return_inverse=True)
    first = torch.zeros(u.numel(), dtype=torch.int64).scatter_(0, inv, own)
    assert torch.equal(first[inv], own)


def test_lpt_place_native_matches_numpy_reference():
    from oni355.ops import native
    from oni355.pipeline import common
    r = np.random.default_rng(3)
    counts = np.sort(r.zipf(1.3, 5000).astype(np.int64))[::-1].copy()
    load0 = r.integers(0, 1000, 8).astype(np.int64)
    l1 = load0.copy()
    own = common.lpt_place(counts, l1)
    l2 = load0.copy()
    ref = np.zeros(counts.size, np.int32)
    for i, c in enumerate(counts):
        k = int(np.argmin(l2))
        l2[k] += c
        ref[i] = k
    assert native.lib().oni_lpt_place is not None
    assert np.array_equal(own, ref) and np.array_equal(l1, l2)


@pytest.mark.parametrize("W", [1, 2, 3, 8])
def test_x01_packed_sum_is_exact(W):
    """Σ over W ranks of packed buffers (int32 wrap-around, as RCCL sums) unpacks to the exact
    per-entry sum whenever every tiny value is within ±O8 and every light value within ±O."""
    from oni355 import ops
    r = np.random.default_rng(W)
    V, KS, tail = 300, 20, 37
    O, O8 = 32767 // W, 127 // W
    perm = r.permutation(V)
    heavy = torch.from_numpy(np.sort(perm[:40]).astype(np.int32))
    tiny = torch.from_numpy(np.sort(perm[40:200]).astype(np.int32))
    light = torch.from_numpy(np.sort(perm[200:]).astype(np.int32))
    n = ops.x01_packed_len(tiny.numel(), light.numel(), heavy.numel(), KS, tail)
    assert n == 160 * KS // 4 + 100 * KS // 2 + 40 * KS + tail
    total = torch.zeros(V * KS + tail, dtype=torch.int64)
    acc = torch.zeros(n, dtype=torch.int64)
    for _ in range(W):
        dn = torch.from_numpy(r.integers(-O, O + 1, V * KS + tail).astype(np.int32))
        rows = dn.view(-1)[: V * KS].view(V, KS)
        rows[heavy.long()] = torch.from_numpy(r.integers(-2**24, 2**24, (heavy.numel(), KS)).astype(np.int32))
        rows[tiny.long()] = torch.from_numpy(r.integers(-O8, O8 + 1, (tiny.numel(), KS)).astype(np.int32))
        total += dn.to(torch.int64)
        out = torch.zeros(n, dtype=torch.int32)
        ops.x01_pack(dn, tiny, light, heavy, KS, V * KS, tail, O8, O, out)
        acc += out.to(torch.int64) & 0xFFFFFFFF
    summed = ((acc + 2**31) % 2**32 - 2**31).to(torch.int32)  # int32 wrap-around sum
    back = torch.zeros(V * KS + tail, dtype=torch.int32)
    ops.x01_unpack(summed, tiny, light, heavy, KS, V * KS, tail, W * O8, W * O, back)
    assert torch.equal(back.to(torch.int64), total)


def _single_worker(rank, world, port, source, n_total, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from oni355.parallel import comm as pc
    from oni355.store.columnar import StringColumn
    comm = pc.init_from_env("cpu") if world > 1 else None
    if source == "dns":
        from oni355.pipeline.dns import run_dns as run
        from oni355.synth.dns import generate_dns as gen
        K = 10
    else:
        from oni355.pipeline.proxy import run_proxy as run
        from oni355.synth.proxy import generate_proxy as gen
        K = 20
    cols = gen(n_total, seed=4).cols
    per = n_total // world
    lo = rank * per
    hi = n_total if rank == world - 1 else lo + per
    cols = {k: (v.slice(lo, hi) if isinstance(v, StringColumn) else v[lo:hi]) for k, v in cols.items()
            if not k.startswith("_")}
    res = run(cols, K=K, sweeps=4, maxresults=120, device="cpu", comm=comm, row_offset=lo)
    from oni355.io import results as rio
    text = rio.render_result(source, cols, res, lo, comm).blob  # rows rendered where they live, gathered
    if rank == 0:
        out_q.put((res.rows, res.scores, res.words, text))
    if comm is not None:
        comm.barrier()
        pc.shutdown()


@pytest.mark.parametrize("source", ["dns", "proxy"])
def test_dns_proxy_dp_matches_single_process(source):
    """DNS / proxy (one token per event, owner-side scoring, result words gathered from the rank
    that holds each row) on 2 gloo ranks == one process: rows, scores, words and the rendered CSV
    rows (each formatted on the rank holding the raw row, gathered as one byte tensor)."""
    ctx = mp.get_context("spawn")
    out = []
    for world in (1, 2):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_single_worker, args=(r, world, port, source, 5000, q)) for r in range(world)]
        for p in procs:
            p.start()
        out.append(q.get(timeout=600))
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
    (r1, s1, w1, t1), (r2, s2, w2, t2) = out
    assert r1.size > 0
    assert np.array_equal(r1, r2) and np.array_equal(s1, s2) and np.array_equal(w1, w2)
    assert t1 == t2 and t1.count(b"\n") == r1.size  # the CSV rows, gathered from both ranks


def _forced_real_worker(port, n_total, out_q, env):
    os.environ.update(env)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.set_num_threads(1)
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    comm = pc.init_from_env("cpu")
    assert comm.dist and comm.world == 1 and comm.live == (env.get("ONI_COMM_REAL") == "1")
    res = run_flow(dict(generate_flows(n_total, seed=11).cols), K=20, sweeps=4, maxresults=150, device="cpu",
                   comm=comm)
    out_q.put((res.rows, res.scores, res.src_scores, res.dst_scores, res.stats["loglik"],
               res.lda.model._x01 is not None, res.lda.model._inplace_ok))
    comm.barrier()
    pc.shutdown()


@pytest.mark.parametrize("env", [{"ONI_FORCE_DIST": "1", "ONI_COMM_REAL": "1"},
                                 {"ONI_FORCE_DIST": "1", "ONI_COMM_REAL": "1", "ONI_X01_PACK": "1"}])
def test_forced_real_one_rank_group_matches_single_process(env):
    """ONI_COMM_REAL=1: a 1-rank process group runs every collective for real (X01 on the Δ
    buffer -- packed too --, the vocabulary gather, the routing all-to-all, the result gather);
    the run stays bitwise equal to the plain single process, and the in-place apply (which would
    bypass the Δ buffer the all-reduce reads) is off."""
    n = 6000
    one = _run_world(1, n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_real_worker, args=(_free_port(), n, q, env))
    p.start()
    res = q.get(timeout=600)
    p.join(timeout=120)
    assert p.exitcode == 0
    for a, b in zip(one[:4], res[:4]):
        assert np.array_equal(a, b)
    assert one[4] == pytest.approx(res[4], rel=1e-9)
    assert res[5] == (env.get("ONI_X01_PACK") == "1")
    assert res[6] is False


class _FakeGraph:
    def replay(self):
        raise AssertionError("a graph was replayed although another rank's capture failed")


def _vote_worker(rank, world, port, n_total, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from oni355.models.gibbs import GibbsLDA
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows

    # CPU stand-ins for HIP graph capture: rank 1's capture raises, rank 0's "succeeds"
    def fake_capture(self, mode):
        if rank == 1:
            raise RuntimeError("hipErrorStreamCaptureInvalidated (simulated)")
        entry = (_FakeGraph(), (self.a, self.b, self.cn))
        self._graphs[(mode, self._acc, self._lag_live)] = entry
        return entry
    GibbsLDA._graphable = lambda self: not getattr(self, "_graph_off", False)
    GibbsLDA._capture = fake_capture
    comm = pc.init_from_env("cpu")
    day = generate_flows(n_total, seed=11)
    per = n_total // world
    lo = rank * per
    hi = n_total if rank == world - 1 else lo + per
    cols = {k: v[lo:hi] for k, v in day.cols.items()}
    res = run_flow(cols, K=20, sweeps=4, maxresults=150, device="cpu", comm=comm, row_offset=lo)
    fb = res.lda.model.timings.get("graph_fallback")
    got = comm.allgather_var(torch.tensor([1 if fb else 0]))
    if rank == 0:
        out_q.put((res.rows, res.scores, res.src_scores, res.dst_scores, res.stats["loglik"],
                   [int(t[0]) for t in got], res.lda.model.timings.get("graph_replays", 0)))
    comm.barrier()
    pc.shutdown()


def test_capture_failure_on_one_rank_sends_every_rank_to_eager_sweeps():
    """The sweep-graph capture vote (GibbsLDA._capture_agreed): rank 1's capture fails, rank 0's
    succeeds; the MIN all-reduce makes BOTH ranks drop their graphs and sweep eagerly (rank 0's
    graph is never replayed), and the day is still bitwise the single-process day."""
    n = 6000
    one = _run_world(1, n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_vote_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for a, b in zip(one[:4], res[:4]):
        assert np.array_equal(a, b)
    assert one[4] == pytest.approx(res[4], rel=1e-9)
    assert res[5] == [1, 1] and res[6] == 0


def test_agree_is_a_min_vote():
    from oni355.parallel.comm import Comm
    assert Comm().agree(True) and not Comm().agree(False)
