"""Checkpoint/resume (bitwise, also across rank counts) and fault injection."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oni355.pipeline.flow import run_flow
from oni355.synth.flow import generate_flows
from oni355.utils import fault
from oni355.utils.checkpoint import Checkpointer


def _day():
    return generate_flows(5000, seed=21)


def test_resume_is_bitwise(tmp_path):
    day = _day()
    full = run_flow(day.cols, K=20, sweeps=8, maxresults=60, device="cpu")
    ck = Checkpointer(str(tmp_path / "ck"), every=3)
    part = run_flow(day.cols, K=20, sweeps=5, maxresults=60, device="cpu", ckpt=ck)  # saves at sweep 3
    assert ck.manifest()["sweep"] == 3
    res = run_flow(day.cols, K=20, sweeps=8, maxresults=60, device="cpu", ckpt=Checkpointer(str(tmp_path / "ck"), 3))
    assert np.array_equal(full.rows, res.rows) and np.array_equal(full.scores, res.scores)
    assert part.lda.model.sweeps_done == 5


def test_fault_injection_then_resume(tmp_path, monkeypatch):
    day = _day()
    full = run_flow(day.cols, K=20, sweeps=6, maxresults=40, device="cpu")
    ck = str(tmp_path / "ck")
    monkeypatch.setenv("ONI_FAULT", "rank:0,sweep:4,kind:raise")
    with pytest.raises(fault.InjectedFault):
        run_flow(day.cols, K=20, sweeps=6, maxresults=40, device="cpu", ckpt=Checkpointer(ck, every=2))
    monkeypatch.delenv("ONI_FAULT")
    assert Checkpointer(ck).manifest()["sweep"] == 4
    res = run_flow(day.cols, K=20, sweeps=6, maxresults=40, device="cpu", ckpt=Checkpointer(ck, every=2))
    assert np.array_equal(full.rows, res.rows) and np.array_equal(full.scores, res.scores)


def test_fault_spec_parse():
    assert fault.parse("rank:2,sweep:7,kind:exit") == {"rank": 2, "sweep": 7, "kind": "exit"}
    assert fault.parse("") is None


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, ckdir, sweeps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from oni355.parallel import comm as pc
    comm = pc.init_from_env("cpu")
    day = _day()
    n = day.n
    per = n // world
    lo = rank * per
    hi = n if rank == world - 1 else lo + per
    cols = {k: v[lo:hi] for k, v in day.cols.items()}
    res = run_flow(cols, K=20, sweeps=sweeps, maxresults=50, device="cpu", comm=comm, row_offset=lo,
                   ckpt=Checkpointer(ckdir, every=2, comm=comm))
    if rank == 0:
        q.put((res.rows, res.scores))
    comm.barrier()
    pc.shutdown()


def test_resume_on_different_rank_count(tmp_path):
    ctx = mp.get_context("spawn")
    ck = str(tmp_path / "ck")
    # 2 ranks train 4 sweeps (checkpoints at 2 and 4) ...
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, ck, 4, q)) for r in range(2)]
    [p.start() for p in ps]
    q.get(timeout=300)
    [p.join(timeout=60) for p in ps]
    assert Checkpointer(ck).manifest() == {"sweep": 4, "world": 2, "ident": Checkpointer(ck).manifest()["ident"]}
    # ... and 1 rank resumes to 6: must equal an uninterrupted single-rank 6-sweep run
    resumed = run_flow(_day().cols, K=20, sweeps=6, maxresults=50, device="cpu", ckpt=Checkpointer(ck, every=2))
    full = run_flow(_day().cols, K=20, sweeps=6, maxresults=50, device="cpu")
    assert np.array_equal(full.rows, resumed.rows) and np.array_equal(full.scores, resumed.scores)


def test_watchdog_fires_and_kick_defers():
    import time

    from oni355.utils.fault import Watchdog
    fired = []
    w = Watchdog(0.2, on_timeout=lambda: fired.append(time.monotonic()))
    for _ in range(5):
        time.sleep(0.08)
        w.kick()
    assert not fired
    time.sleep(0.6)
    assert fired
    w.close()


def test_invariant_checks_run_and_catch_corruption():
    import numpy as np
    import pytest
    import torch

    from oni355.models.corpus import build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    r = np.random.default_rng(1)
    lens = r.integers(1, 100, 30)
    c = build_corpus(torch.from_numpy(np.repeat(np.arange(30), lens)), torch.from_numpy(r.integers(0, 25, int(lens.sum()))),
                     30, 25, torch.arange(30, dtype=torch.int32), 1, L=64)
    m = GibbsLDA(c, GibbsConfig(K=20, seed=1, check_invariants=True))
    m.initialize()
    m.sweep(3)
    m.nwk[0, 0] -= 1
    with pytest.raises(AssertionError):
        m.check_invariants()
