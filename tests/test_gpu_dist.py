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


def _forced_rccl_worker(port, n_total, sweeps, out_q, heavy=0.0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ONI_FORCE_DIST="1",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    if heavy:
        # cut the heavy IP even in the 1-rank group (pieces of 1/8 of the day's tokens)
        os.environ.update(ONI_SPLIT_MIN_WORLD="1", ONI_SPLIT_DEN="8")
    os.environ.pop("WORLD_SIZE", None)
    os.environ.pop("ONI_DIST_BACKEND", None)
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    comm = pc.init_from_env("cuda")
    assert comm.dist and comm.backend == "nccl" and comm.graph_capturable()
    res = run_flow(_flow_cols(n_total, heavy), K=20, sweeps=sweeps, maxresults=200, device="cuda:0", comm=comm)
    m = res.lda.model
    c = res.lda.corpus
    out_q.put((res.rows, res.scores, res.stats["loglik"], m.timings.get("graph_replays", 0), m.allreduce_ms_per_sweep(),
               m.allreduce_bytes_per_sweep(), int(c.split["n_split"]) if c.split is not None else 0))
    comm.barrier()
    pc.shutdown()


@pytest.mark.parametrize("heavy", [0.0, 0.30])
def test_forced_rccl_sweeps_replay_from_graphs_bitwise(gpu, heavy):
    """A 1-rank RCCL process group (ONI_FORCE_DIST=1): every data-parallel code path (placement,
    routing, split pieces, owner scoring, result merge) runs, the sweeps replay from HIP graphs, and
    the run stays bitwise equal to the world=1 run -- also with a 30 % IP cut into pieces whose
    Δn_dk rows travel in the X01 buffer. (A 1-rank group's collectives are the identity: no RCCL
    kernel runs, comm.Comm.)"""
    n, sweeps = 20_000, 8
    from oni355.pipeline.flow import run_flow
    plain = run_flow(_flow_cols(n, heavy), K=20, sweeps=sweeps, maxresults=200, device="cuda:0")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_rccl_worker, args=(_free_port(), n, sweeps, q, heavy))
    p.start()
    try:
        rows, scores, ll, n_graphs, ar_ms, ar_bytes, n_split = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.exitcode is None:
            p.kill()
    assert p.exitcode == 0
    assert n_graphs >= 1, "DP sweeps were not captured into a HIP graph"
    assert ar_ms is not None and ar_bytes > 0
    assert np.array_equal(plain.rows, rows) and np.array_equal(plain.scores, scores)
    assert plain.stats["loglik"] == ll
    assert (n_split >= 1) == (heavy > 0)
