"""Multi-day product path (pipeline.daily, ``oni-ml <range>`` / ``--follow``): days stream from the
columnar store with loading overlapped, and every day's results equal a single-day run."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oni355.store import columnar

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATES = ["20160708", "20160709", "20160710"]


def _store(tmp_path, source, n=3000, ipv6=0.0):
    root = str(tmp_path / "store")
    for i, d in enumerate(DATES):
        if source == "flow":
            from oni355.synth.flow import generate_flows
            cols = generate_flows(n, seed=20 + i, ipv6_frac=ipv6).cols
        elif source == "dns":
            from oni355.synth.dns import generate_dns
            cols = {k: v for k, v in generate_dns(n, seed=20 + i).cols.items() if not k.startswith("_")}
        else:
            from oni355.synth.proxy import generate_proxy
            cols = generate_proxy(n, seed=20 + i).cols
        columnar.write_day(root, source, d, cols)
    return root


def _cli(args, env=None):
    r = subprocess.run([sys.executable, "-m", "oni355.cli.ml", *args], cwd=ROOT, capture_output=True, text=True,
                       timeout=900, env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("source", ["flow", "dns", "proxy"])
def test_date_range_equals_single_day_runs(tmp_path, source):
    root = _store(tmp_path, source, ipv6=0.2 if source == "flow" else 0.0)
    conf = str(tmp_path / "none.conf")
    common = ["--data-root", root, "--device", "cpu", "--sweeps", "4", "--config", conf, "--topics", "10"]
    multi = str(tmp_path / "multi")
    out = json.loads(_cli([f"{DATES[0]}-{DATES[-1]}", source, "1.0", "200", "--lpath", multi, *common]))
    assert out["days"] == DATES and out["events"] == 3 * 3000
    for d in DATES:
        single = str(tmp_path / f"single_{d}")
        _cli([d, source, "1.0", "200", "--lpath", single, "--quiet", *common])
        a = open(os.path.join(multi, source, d, f"{source}_results.csv")).read()
        b = open(os.path.join(single, source, d, f"{source}_results.csv")).read()
        assert a == b and a.count("\n") == 201
        rec = [json.loads(x) for x in open(os.path.join(multi, source, d, "metrics.jsonl"))]
        assert rec[-1]["event"] == "oni-ml-day" and rec[-1]["date"] == d


def test_follow_picks_up_complete_days(tmp_path):
    from oni355.parallel.comm import Comm
    from oni355.pipeline.daily import run_days
    root = _store(tmp_path, "flow")
    os.remove(os.path.join(columnar.day_dir(root, "flow", DATES[2]), "_SUCCESS"))  # still ingesting
    assert columnar.days(root, "flow") == DATES[:2]
    kw = dict(K=10, sweeps=3, tol=1.0, maxresults=50, device="cpu")
    recs = run_days("flow", [DATES[0]], root, str(tmp_path / "lp"), Comm(), kw, "cpu", follow=True, poll_s=0.05,
                    idle_exit_s=0.3)
    assert [r["date"] for r in recs] == DATES[:2]
    assert not os.path.exists(os.path.join(tmp_path, "lp", "flow", DATES[2]))


def test_mmap_read_day_is_zero_copy_and_equal(tmp_path):
    root = _store(tmp_path, "proxy")
    a = columnar.read_day(root, "proxy", DATES[0], row_range=(100, 900))
    b = columnar.read_day(root, "proxy", DATES[0], row_range=(100, 900), mmap=True)
    assert isinstance(b["duration"], np.memmap)
    for k, v in a.items():
        if hasattr(v, "offsets"):
            assert v.to_list() == b[k].to_list()
        else:
            assert np.array_equal(v, b[k])


def _follow_worker(rank, world, port, root, out_q):
    import os as _os
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                       LOCAL_RANK=str(rank))
    from oni355.parallel import comm as pc
    from oni355.pipeline.daily import _next_days
    comm = pc.init_from_env("cpu")
    # rank 1's clock says "idle" at once, rank 0's only on the second pass: every rank must leave
    # on rank 0's decision, in the same pass
    passes = 0
    while True:
        passes += 1
        _, stop = _next_days(root, "flow", "99999999", comm, idle=(rank == 1) or passes >= 2)
        if stop:
            break
    out_q.put((rank, passes))
    comm.barrier()
    pc.shutdown()


def test_follow_idle_exit_is_decided_by_rank0(tmp_path):
    """the --follow idle exit comes from rank 0 with the day list, not each rank's clock."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_follow_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == [(0, 2), (1, 2)]
