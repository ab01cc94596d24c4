"""Data parallel at 8 ranks without a GPU cluster (gloo, CPU tensors): every source's day on 8
ranks reproduces the single-process run bit for bit; a day with one IP holding 30 % of the tokens
is cut into chunk-aligned pieces (pipeline.common.SplitPlan) and balances within 10 % across the
8 ranks; analyst feedback enters the corpus once (DUPFACTOR, not world × DUPFACTOR); checkpoints
of a run with split documents resume on another rank count."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

HEAVY_IP = 0x0A0B0C0D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _slice_cols(cols, lo, hi):
    from oni355.store.columnar import StringColumn
    return {k: (v.slice(lo, hi) if isinstance(v, StringColumn) else v[lo:hi]) for k, v in cols.items()
            if not k.startswith("_")}


def _day(source, n, heavy, wide=False):
    if source == "flow":
        from oni355.synth.flow import generate_flows
        day = generate_flows(n, seed=11, wide_vocab=wide)
        cols = dict(day.cols)
        if heavy:
            r = np.random.default_rng(5)
            sip = np.asarray(cols["sip"]).copy()
            sip[r.random(n) < 2 * heavy] = HEAVY_IP  # 2 tokens per flow: 2·heavy of the flows
            cols["sip"] = sip
        return cols
    if source == "dns":
        from oni355.synth.dns import generate_dns
        return dict(generate_dns(n, seed=4).cols)
    from oni355.synth.proxy import generate_proxy
    return dict(generate_proxy(n, seed=4).cols)


def _worker(rank, world, port, job, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.update(job.get("env", {}))
    torch.set_num_threads(1)
    from oni355.parallel import comm as pc
    comm = pc.init_from_env("cpu") if world > 1 else None
    source, n = job["source"], job["n"]
    cols = _day(source, n, job.get("heavy", 0.0), job.get("wide", False))
    per = n // world
    lo = rank * per
    hi = n if rank == world - 1 else lo + per
    mine = _slice_cols(cols, lo, hi)
    fb = None
    if job.get("feedback"):
        fb = _slice_cols(cols, 0, 40)  # analyst sev=3 rows (same file on every rank)
    kw = dict(K=job.get("K", 20), sweeps=job.get("sweeps", 4), maxresults=150, device="cpu", comm=comm, row_offset=lo,
              feedback=fb, dupfactor=50)
    ck = None
    if job.get("ckpt"):
        from oni355.utils.checkpoint import Checkpointer
        ck = Checkpointer(job["ckpt"], every=job.get("ckpt_every", 0), comm=comm)
        kw["ckpt"] = ck
    if source == "flow":
        from oni355.pipeline.flow import run_flow
        res = run_flow(mine, **kw)
    elif source == "dns":
        from oni355.pipeline.dns import run_dns
        res = run_dns(mine, **kw)
    else:
        from oni355.pipeline.proxy import run_proxy
        res = run_proxy(mine, **kw)
    c = res.lda.corpus
    loads = [c.T]
    n_split = int(c.split["n_split"]) if c.split is not None else 0
    if comm is not None:
        loads = [int(x) for x in torch.cat(comm.allgather_var(torch.tensor([c.T]))).tolist()]
    m = res.lda.model
    x = m._x01
    x01 = None if x is None else dict(tiny=int(x["tiny"].numel()), light=int(x["light"].numel()),
                                      heavy=int(x["heavy"].numel()), bytes=m.allreduce_bytes_per_sweep(),
                                      dense_bytes=int(m.dn[0].numel() * 4))
    if rank == 0:
        out_q.put(dict(rows=res.rows, scores=res.scores, loglik=res.stats["loglik"], loads=loads, n_split=n_split,
                       sweeps=m.sweeps_done, x01=x01, qpf=m.qpf))
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
    assert a["rows"].size > 0
    assert np.array_equal(a["rows"], b["rows"])
    assert np.array_equal(a["scores"], b["scores"])
    assert a["loglik"] == pytest.approx(b["loglik"], rel=1e-9)


def test_split_placement_balances_a_30pct_document():
    """8 ranks, one IP with 30 % of the tokens: pieces + LPT keep every rank within 10 % of the
    mean sampling load (whole-document placement leaves that rank at 2.4× the mean)."""
    from oni355.pipeline import common

    class _Comm:
        world = 8
        dist = live = True

        def allgather_var(self, t):
            return [t]

        def allreduce_(self, t):
            return t

        def allreduce_scalar(self, x):
            return x

    r = np.random.default_rng(0)
    keys = r.zipf(1.3, 600_000).astype(np.int64) * 7919 % (2**32)
    keys[r.random(keys.size) < 0.30] = HEAVY_IP
    keys = torch.from_numpy(keys)
    w = torch.ones_like(keys)
    own, plan = common.place_docs(keys, w, _Comm(), split_L=128)
    assert plan is not None and plan.n >= 1
    assert bool((plan.keys == HEAVY_IP).any())
    heavy = torch.isin(keys, plan.keys)  # the 30 % IP, and any other document above 1/16 of the day
    load = torch.bincount(own[~heavy], minlength=8).to(torch.float64)
    for j, p0, p1, o in zip(plan.piece_doc, plan.piece_p0, plan.piece_p1, plan.piece_owner):
        load[int(o)] += int(p1 - p0)
    assert int(load.sum()) == keys.numel()
    assert float(load.max() / load.mean()) < 1.10
    assert np.all(plan.piece_p0 % 128 == 0)
    whole = common.place_docs(keys, w, _Comm())
    wl = torch.bincount(whole, minlength=8).to(torch.float64)
    assert float(wl.max() / wl.mean()) > 2.0


def test_flow_world8_heavy_ip_bitwise_and_balanced():
    job = dict(source="flow", n=16000, heavy=0.30)
    one = _run(1, job)
    eight = _run(8, job)
    _same(one, eight)
    assert eight["n_split"] >= 1
    loads = np.asarray(eight["loads"], np.float64)
    assert loads.max() / loads.mean() < 1.10, loads


def test_mh_sampler_world4_heavy_ip_bitwise():
    """The MH sampler (one-lane units, alias proposals; heavy IP cut across ranks) gives the
    world-1 chain on 4 gloo ranks."""
    job = dict(source="flow", n=12000, heavy=0.30, K=40, sweeps=5, env={"ONI_SAMPLER": "mh"})
    one = _run(1, job)
    four = _run(4, job)
    _same(one, four)
    assert four["n_split"] >= 1 and one["qpf"] == four["qpf"] == 4


def test_mh_after_dense_burn_world4_bitwise():
    """An MH model's first sweeps run the dense kernel on a corpus of the dense tiling, then the
    chain moves to the MH corpus through its canonical z (pipeline.common.build_and_train): the
    same chain on 1 and 4 ranks (heavy IP cut across ranks), and different from pure MH."""
    job = dict(source="flow", n=12000, heavy=0.30, K=40, sweeps=6, env={"ONI_SAMPLER": "mh", "ONI_MH_BURN": "3"})
    one = _run(1, job)
    four = _run(4, job)
    _same(one, four)
    assert four["n_split"] >= 1 and one["qpf"] == four["qpf"] == 4 and four["sweeps"] == 6
    pure = _run(1, dict(job, env={"ONI_SAMPLER": "mh", "ONI_MH_BURN": "0"}))
    assert pure["qpf"] == 4 and pure["loglik"] != one["loglik"]


@pytest.mark.parametrize("w_save,w_resume,at", [(3, 1, 2), (1, 2, 4)])
def test_mh_burn_checkpoint_resumes_on_another_world(tmp_path, w_save, w_resume, at):
    """A checkpoint inside the dense burn-in (sweep 2 of 3) or after the hand-over (sweep 4) on
    w_save ranks resumes on w_resume ranks, equal to an uninterrupted single-rank run."""
    ck = str(tmp_path / "ck")
    base = dict(source="flow", n=8000, heavy=0.30, K=40, env={"ONI_SAMPLER": "mh", "ONI_MH_BURN": "3"})
    ref = _run(1, dict(base, sweeps=6))
    first = _run(w_save, dict(base, sweeps=at, ckpt=ck, ckpt_every=at))
    assert first["sweeps"] == at
    resumed = _run(w_resume, dict(base, sweeps=6, ckpt=ck, ckpt_every=0))
    assert resumed["sweeps"] == 6
    _same(ref, resumed)


@pytest.mark.parametrize("source", ["dns", "proxy"])
def test_dns_proxy_world8_bitwise(source):
    job = dict(source=source, n=6000, K=10 if source == "dns" else 20)
    _same(_run(1, job), _run(8, job))


@pytest.mark.parametrize("source", ["flow", "dns", "proxy"])
def test_feedback_enters_the_corpus_once_on_any_world(source):
    job = dict(source=source, n=5000, feedback=True, K=10 if source == "dns" else 20)
    one = _run(1, job)
    two = _run(2, job)
    _same(one, two)


@pytest.mark.parametrize("w_save,w_resume", [(3, 1), (1, 3)])
def test_split_checkpoint_resumes_on_another_world(tmp_path, w_save, w_resume):
    """Sweeps 1-2 on w_save ranks (heavy IP cut into pieces when w_save > 1), checkpoint, sweeps
    3-4 on w_resume ranks == 4 uninterrupted sweeps on one rank."""
    ck = str(tmp_path / "ck")
    base = dict(source="flow", n=8000, heavy=0.30)
    ref = _run(1, dict(base, sweeps=4))
    first = _run(w_save, dict(base, sweeps=2, ckpt=ck, ckpt_every=2))
    assert first["sweeps"] == 2
    if w_save > 1:
        assert first["n_split"] >= 1
    resumed = _run(w_resume, dict(base, sweeps=4, ckpt=ck, ckpt_every=0))
    assert resumed["sweeps"] == 4
    _same(ref, resumed)


@pytest.mark.parametrize("w_save,w_resume", [(3, 1), (1, 2)])
def test_checkpoint_inside_averaging_window_resumes_on_another_world(tmp_path, w_save, w_resume):
    """A checkpoint taken inside the posterior-averaging window (16 sweeps: samples at 14 and 16)
    on w_save ranks resumes on w_resume ranks; the averaged θ/φ -- hence the scored rows -- equal
    an uninterrupted single-rank run bit for bit."""
    ck = str(tmp_path / "ck")
    base = dict(source="flow", n=8000, heavy=0.30, sweeps=16)
    ref = _run(1, base)
    first = _run(w_save, dict(base, ckpt=ck, ckpt_every=14))
    assert first["sweeps"] == 16
    resumed = _run(w_resume, dict(base, ckpt=ck, ckpt_every=0))
    assert resumed["sweeps"] == 16
    _same(ref, resumed)


def test_realistic_vocab_world8_packed_x01_bitwise():
    """A realistic-vocabulary flow day on 8 ranks with the packed X01 payload (8-bit tiny words,
    16-bit light words, int32 heavy words): bit for bit the single-rank run, at a fraction of the
    dense payload."""
    job = dict(source="flow", n=12000, wide=True, env={"ONI_X01_PACK": "1"})
    one = _run(1, job)
    eight = _run(8, job)
    _same(one, eight)
    x = eight["x01"]
    assert x is not None and x["tiny"] > 0
    assert x["bytes"] < 0.4 * x["dense_bytes"], x


def test_document_above_the_split_threshold_is_proposed_whatever_H():
    """proposals were only the documents above 1/H of a rank's tokens, which covers every
    document above the split threshold 1/(SPLIT_DEN·W) of the day only while SPLIT_DEN·W ≤ H. With
    H = 4 and SPLIT_DEN·W = 8 an IP with 18 % of the tokens (above 1/8, below 1/4 of each rank's) is
    still cut into pieces, and the day stays bitwise the single-process day."""
    env = {"ONI_HEAVY_DOCS_PER_RANK": "4", "ONI_SPLIT_DEN": "2"}
    job = dict(source="flow", n=8000, heavy=0.18, env=env)
    one = _run(1, job)
    four = _run(4, job)
    assert four["n_split"] >= 1
    assert np.array_equal(one["rows"], four["rows"]) and np.array_equal(one["scores"], four["scores"])
