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


def _worker(rank, world, port, n_total, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", ONI_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    torch.set_num_threads(2)
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    comm = pc.init_from_env("cuda")
    day = generate_flows(n_total, seed=11)
    per = n_total // world
    lo = rank * per
    hi = n_total if rank == world - 1 else lo + per
    cols = {k: v[lo:hi] for k, v in day.cols.items()}
    res = run_flow(cols, K=20, sweeps=6, maxresults=200, device="cuda:0", comm=comm, row_offset=lo)
    if rank == 0:
        out_q.put((res.rows, res.scores, res.src_scores, res.dst_scores, res.stats["loglik"]))
    comm.barrier()
    pc.shutdown()


def _run_world(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
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
