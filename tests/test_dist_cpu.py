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


def _worker(rank, world, port, n_total, out_q):
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


def _run_world(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_dp_matches_single_process(world):
    n = 6000
    one = _run_world(1, n)
    many = _run_world(world, n)
    assert np.array_equal(one[0], many[0])
    assert np.array_equal(one[1], many[1])
    assert np.array_equal(one[2], many[2]) and np.array_equal(one[3], many[3])
    assert one[4] == pytest.approx(many[4], rel=1e-9)
