"""Data-parallel sampler on the real HIP kernels with several ranks sharing the one GPU.

SURVEY.md §4.3 "DP without a cluster": RCCL needs one GPU per rank, so the ranks here use gloo
(``ONI_DIST_BACKEND=gloo``; Comm routes device collectives through host copies) while every
kernel — wordify, quantile cuts, corpus build, Gibbs sweeps, Δn_wk apply, scoring, top-N — runs on
the MI355X. The DP design makes each sample independent of the rank count, so 2 and 3 ranks must
reproduce the single-process top-N rows and scores bitwise.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


HEAVY_IP = 0x0A0B0C0D


def _flow_cols(n_total, heavy):
    from oni355.synth.flow import generate_flows
    cols = dict(generate_flows(n_total, seed=11).cols)
    if heavy:
        sip = np.asarray(cols["sip"]).copy()
        sip[np.random.default_rng(5).random(n_total) < 2 * heavy] = HEAVY_IP  # heavy share of the tokens
        cols["sip"] = sip
    return cols


def _worker(rank, world, port, n_total, out_q, heavy=0.0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), ONI_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    torch.set_num_threads(2)
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    comm = pc.init_from_env("cuda")
    day_cols = _flow_cols(n_total, heavy)
    per = n_total // world
    lo = rank * per
    hi = n_total if rank == world - 1 else lo + per
    cols = {k: v[lo:hi] for k, v in day_cols.items()}
    res = run_flow(cols, K=20, sweeps=6, maxresults=200, device="cuda:0", comm=comm, row_offset=lo)
    c = res.lda.corpus
    if rank == 0:
        out_q.put((res.rows, res.scores, res.src_scores, res.dst_scores, res.stats["loglik"],
                   int(c.split["n_split"]) if c.split is not None else 0))
    comm.barrier()
    pc.shutdown()


def _run_world(world, n_total, heavy=0.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q, heavy)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_dp_ranks_sharing_gpu_match_single_process(gpu, world):
    n = 20_000
    one = _run_world(1, n)
    many = _run_world(world, n)
    assert len(one[0]) > 0
    assert np.array_equal(one[0], many[0])
    assert np.array_equal(one[1], many[1])
    assert np.array_equal(one[2], many[2]) and np.array_equal(one[3], many[3])
    assert one[4] == pytest.approx(many[4], rel=1e-9)


def test_dp_ranks_sharing_gpu_heavy_ip_cut_into_pieces(gpu):
    """One IP with 30 % of the tokens on 3 ranks: its pieces are sampled on the GPU by every rank
    against the global n_dk row (Δ rows in the X01 buffer), bitwise equal to one process."""
    n = 20_000
    one = _run_world(1, n, heavy=0.30)
    three = _run_world(3, n, heavy=0.30)
    assert three[5] >= 1 and one[5] == 0
    for a, b in zip(one[:4], three[:4]):
        assert np.array_equal(a, b)
    assert one[4] == pytest.approx(three[4], rel=1e-9)


def _forced_rccl_worker(port, n_total, sweeps, out_q, heavy=0.0, env=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ONI_FORCE_DIST="1",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    os.environ.update(env or {})
    if heavy:
        # cut the heavy IP even in the 1-rank group (pieces of 1/8 of the day's tokens)
        os.environ.update(ONI_SPLIT_MIN_WORLD="1", ONI_SPLIT_DEN="8")
    os.environ.pop("WORLD_SIZE", None)
    os.environ.pop("ONI_DIST_BACKEND", None)
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    comm = pc.init_from_env("cuda")
    assert comm.dist and comm.backend == "nccl" and comm.graph_capturable()
    assert comm.live == (os.environ.get("ONI_COMM_REAL") == "1")
    res = run_flow(_flow_cols(n_total, heavy), K=20, sweeps=sweeps, maxresults=200, device="cuda:0", comm=comm)
    m = res.lda.model
    c = res.lda.corpus
    out_q.put((res.rows, res.scores, res.stats["loglik"], m.timings.get("graph_replays", 0), m.allreduce_ms_per_sweep(),
               m.allreduce_bytes_per_sweep(), int(c.split["n_split"]) if c.split is not None else 0,
               m._x01 is not None, m.timings.get("graph_fallback")))
    comm.barrier()
    pc.shutdown()


def _forced(n, sweeps, heavy, env):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_rccl_worker, args=(_free_port(), n, sweeps, q, heavy, env))
    p.start()
    try:
        out = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.exitcode is None:
            p.kill()
    assert p.exitcode == 0
    return out


REAL = {"ONI_COMM_REAL": "1"}


@pytest.mark.parametrize("heavy,env", [(0.0, REAL), (0.30, REAL), (0.0, {**REAL, "ONI_X01_PACK": "1"}),
                                       (0.30, {**REAL, "ONI_X01_PACK": "1"}), (0.0, {})])
def test_forced_rccl_sweeps_replay_from_graphs_bitwise(gpu, heavy, env):
    """A 1-rank RCCL process group (ONI_FORCE_DIST=1) with ONI_COMM_REAL=1: every collective runs
    on RCCL for real -- the X01 all-reduce (packed, with ONI_X01_PACK=1) inside the captured sweep
    graphs, the routing all-to-all, the vocabulary / split-piece / top-N gathers, the X03 radix
    histogram all-reduces -- with every data-parallel code path around them (placement, routing,
    split pieces whose Δn_dk rows travel in the X01 buffer, owner scoring, result merge). The run
    replays its sweeps from HIP graphs and stays bitwise equal to the world = 1 run; the per-sweep
    X01 time is a real RCCL all-reduce of the same payload. Without ONI_COMM_REAL the 1-rank
    collectives are the identity (the overhead bench's setting) and the run is bitwise too."""
    n, sweeps = 20_000, 8
    from oni355.pipeline.flow import run_flow
    plain = run_flow(_flow_cols(n, heavy), K=20, sweeps=sweeps, maxresults=200, device="cuda:0")
    rows, scores, ll, n_graphs, ar_ms, ar_bytes, n_split, packed, fb = _forced(n, sweeps, heavy, env)
    assert n_graphs >= 1, "DP sweeps were not captured into a HIP graph"
    assert fb is None
    assert ar_bytes > 0
    if env:
        assert ar_ms is not None and ar_ms > 0
        assert packed == (env.get("ONI_X01_PACK") == "1")
    assert np.array_equal(plain.rows, rows) and np.array_equal(plain.scores, scores)
    assert plain.stats["loglik"] == ll
    assert (n_split >= 1) == (heavy > 0)


def test_forced_rccl_capture_failure_falls_back_to_eager_bitwise(gpu):
    """ONI_FAULT=rank:0,kind:capture fails the sweep-graph capture (between capture begin and
    end, with the RCCL all-reduce in the graph): the vote sends the rank to eager sweeps -- the
    same kernels and RCCL calls, no replay -- and the day is still bitwise the plain day."""
    n, sweeps = 20_000, 8
    from oni355.pipeline.flow import run_flow
    plain = run_flow(_flow_cols(n, 0.0), K=20, sweeps=sweeps, maxresults=200, device="cuda:0")
    rows, scores, ll, n_graphs, ar_ms, ar_bytes, n_split, packed, fb = _forced(
        n, sweeps, 0.0, {**REAL, "ONI_X01_PACK": "1", "ONI_FAULT": "rank:0,kind:capture"})
    assert n_graphs == 0 and fb is not None and "injected" in fb
    assert ar_ms is not None and ar_ms > 0  # eager sweeps: HIP events around each real all-reduce
    assert np.array_equal(plain.rows, rows) and np.array_equal(plain.scores, scores)
    assert plain.stats["loglik"] == ll
