"""Lagged X01 (ONI_X01_LAG=1, models/gibbs.py): the Δ all-reduce of sweep s runs on a side stream
during sweep s + 1, so every lagged sweep samples its word side against the global counts one
sweep older than its doc rows, with the word-side exclusion at the token's topic in those counts
(tok_zlag, spec.gibbs_pass). The rule is the same on any number of ranks: world 1, 2, 3 and 8
are bit for bit one chain, with the heavy-IP split pieces and with the packed payload; sweep()
calls end in a drain, so the counts are current between calls (checkpoints, likelihood)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oni355 import ops
from oni355.models.corpus import build_corpus
from oni355.models.gibbs import GibbsConfig, GibbsLDA

LAG = {"ONI_X01_LAG": "1", "ONI_X01_LAG_FROM": "3"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, job, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.update(job.get("env", {}))
    torch.set_num_threads(1)
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    comm = pc.init_from_env("cpu") if world > 1 else None
    n = job["n"]
    cols = dict(generate_flows(n, seed=11, wide_vocab=job.get("wide", False)).cols)
    if job.get("heavy"):
        sip = np.asarray(cols["sip"]).copy()
        sip[np.random.default_rng(5).random(n) < 0.6] = 0x0A0B0C0D
        cols["sip"] = sip
    per = n // world
    lo = rank * per
    hi = n if rank == world - 1 else lo + per
    mine = {k: v[lo:hi] for k, v in cols.items()}
    res = run_flow(mine, K=20, sweeps=job.get("sweeps", 8), maxresults=150, device="cpu", comm=comm, row_offset=lo,
                   eval_every=job.get("eval_every", 0))
    m = res.lda.model
    if rank == 0:
        out_q.put(dict(rows=res.rows, scores=res.scores, loglik=res.stats["loglik"], lag=m._lag_live,
                       chain=dict(m.chain), n_split=int(res.lda.corpus.split["n_split"]) if res.lda.corpus.split
                       is not None else 0, calls=m.timings["allreduce_calls"]))
    if comm is not None:
        comm.barrier()
        pc.shutdown()


def _run(world, job):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, job, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=900)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return res


def _same(a, b):
    assert np.array_equal(a["rows"], b["rows"]) and np.array_equal(a["scores"], b["scores"])
    assert a["loglik"] == pytest.approx(b["loglik"], rel=1e-9)


@pytest.mark.parametrize("world,extra", [(2, {}), (3, {"ONI_X01_PACK": "1", "ONI_X01_LIGHT_MAX": "40"}),
                                         (8, {})])
def test_lagged_chain_is_the_same_on_any_world(world, extra):
    job = dict(n=6000, env={**LAG, **extra}, eval_every=5, sweeps=11)
    one = _run(1, job)
    many = _run(world, job)
    assert one["lag"] and many["lag"] and one["chain"].get("x01_lag") == 1
    _same(one, many)


def test_lagged_chain_with_split_pieces_world3():
    """A 30 % IP cut into pieces: its Δn_dk rows stay synchronous, the word side lags."""
    job = dict(n=6000, heavy=True, env={**LAG, "ONI_SPLIT_DEN": "8"})
    one = _run(1, job)
    three = _run(3, job)
    assert three["n_split"] >= 1
    _same(one, three)


def test_lag_is_a_different_chain_and_off_until_it_starts():
    """Before ONI_X01_LAG_FROM the lag-configured model draws the synchronous chain bit for bit;
    once it lags, the chain differs (the word side is one sweep older)."""
    base = _run(1, dict(n=4000, env={}))
    late = _run(1, dict(n=4000, env={"ONI_X01_LAG": "1", "ONI_X01_LAG_FROM": "1000"}))
    on = _run(1, dict(n=4000, env=LAG))
    _same(base, late)
    assert not late["lag"] and on["lag"]
    assert not np.array_equal(base["scores"], on["scores"])


def _toy(dev, K, seed=3):
    r = np.random.default_rng(seed)
    D, V = 200, 300
    lens = r.zipf(1.6, D).clip(1, 2000)
    lens[0] = 3000
    tdoc = np.repeat(np.arange(D), lens)
    tword = (r.zipf(1.3, tdoc.size) - 1) % V
    keys = torch.from_numpy(((np.arange(D, dtype=np.int64) * 2654435761 + seed) % (2**31 - 1)).astype(np.int32))
    G, _ = ops.choose_tiling(K)
    return build_corpus(torch.from_numpy(tdoc).to(dev), torch.from_numpy(tword).to(dev), D, V, keys.to(dev), G, L=64)


@pytest.mark.gpu
@pytest.mark.parametrize("K,mode,sampler,graph", [(20, "auto", "dense", True), (20, "wdelta", "dense", False),
                                                  (20, "recount", "dense", True), (50, "wdelta", "dense", True),
                                                  (100, "auto", "dense", True), (7, "wdelta", "dense", False),
                                                  (20, "wdelta", "generic", True)])
def test_lagged_kernels_match_the_oracle_bitwise(gpu, monkeypatch, K, mode, sampler, graph):
    """k_gibbs_x1 / k_gibbs_ldsg / k_gibbs with tok_zlag (their LAG variants) against the NumPy
    oracle, bit for bit, across sweep() calls (drains) -- with the side-stream X01 captured into
    the sweep graphs."""
    monkeypatch.setenv("ONI_X01_LAG_FROM", "3")
    cc, cg = _toy(torch.device("cpu"), K), _toy(gpu, K)
    mc = GibbsLDA(cc, GibbsConfig(K=K, seed=77, use_graph=False, count_mode="atomic", sampler="dense", x01_lag=True,
                                  auto_switch=0))
    mg = GibbsLDA(cg, GibbsConfig(K=K, seed=77, use_graph=graph, count_mode=mode, sampler=sampler, x01_lag=True,
                                  auto_switch=5 if mode == "auto" else 0))
    for m in (mc, mg):
        m.initialize()
    for n in (4, 6, 3):
        mc.sweep(n)
        mg.sweep(n)
        assert mg._lag_live and mc._lag_live
        for a, b in ((mc.tok_z, mg.tok_z), (mc.tok_zlag, mg.tok_zlag), (mc.nwk, mg.nwk), (mc.nk_cur, mg.nk_cur),
                     (mc.ndk_cur, mg.ndk_cur), (mc.q, mg.q), (mc.qfix, mg.qfix)):
            assert torch.equal(a, b.cpu())
    if graph:
        assert mg.timings.get("graph_replays", 0) >= 1
    mg.check_invariants()
    mg.close()


def test_lagged_chain_resumes_bitwise_from_a_checkpoint(tmp_path, monkeypatch):
    """sweep() calls end in a drain, and the lag starts at a fixed sweep: a run checkpointed inside
    the lagged stretch and resumed in a fresh model is bit for bit the uninterrupted run."""
    monkeypatch.setenv("ONI_X01_LAG_FROM", "3")
    from oni355.utils.checkpoint import Checkpointer
    cpu = torch.device("cpu")

    def model():
        m = GibbsLDA(_toy(cpu, 20), GibbsConfig(K=20, seed=4, x01_lag=True, sampler="dense"))
        return m
    a = model()
    a.initialize()
    for n in (5, 4, 4):
        a.sweep(n)
    b = model()
    b.initialize()
    b.sweep(5)
    b.sweep(4)
    ck = Checkpointer(str(tmp_path))
    ck.save(b)
    c = model()
    assert ck.restore(c) == 9
    c.sweep(4)
    assert torch.equal(a.canonical_z(), c.canonical_z())
    assert torch.equal(a.nwk, c.nwk) and torch.equal(a.ndk_cur, c.ndk_cur) and torch.equal(a.q, c.q)
