"""IPv6 flows end to end: nfcapd / nfdump-CSV decoders carry the 16-byte addresses (text columns
sip6/dip6), the pipeline keys every distinct IPv6 address exactly (240.0.0.0/4 + dictionary rank,
identical on every rank), results print the IPv6 text, and analyst feedback on an IPv6 row
reaches the right document."""
import csv
import os

import numpy as np
import pytest

from oni355.io import decoders, nfcapd
from oni355.pipeline.flow import V6_KEY_BASE, run_flow, with_ipv6_keys
from oni355.synth.flow import generate_flows


def _day(n=4000):
    return generate_flows(n, seed=13, ipv6_frac=0.3)


def test_decoders_round_trip_ipv6(tmp_path):
    day = _day()
    n6 = sum(1 for t in day.cols["sip6"].to_list() if t)
    assert 0 < n6 < day.n
    for fmt in ("nfcapd", "csv"):
        p = str(tmp_path / f"d.{fmt}")
        if fmt == "nfcapd":
            nfcapd.write_nfcapd(p, day.cols)
            got = nfcapd.read_nfcapd(p)
        else:
            decoders.write_flow_csv(p, day.cols)
            got, bad = decoders.read_flow_csv(p)
            assert bad == 0
        for c in ("sip6", "dip6"):
            assert got[c].to_list() == day.cols[c].to_list(), (fmt, c)
        assert np.array_equal(got["sip"], day.cols["sip"]) and np.array_equal(got["dport"], day.cols["dport"])


def test_ipv6_keys_exact_and_disjoint_from_ipv4():
    day = _day()
    k = with_ipv6_keys(day.cols)
    v6 = np.array([bool(t) for t in day.cols["sip6"].to_list()])
    assert np.all(k["sip"][v6] >= V6_KEY_BASE) and np.all(k["sip"][~v6] < V6_KEY_BASE)
    # same text <-> same key, across both endpoints
    txt = day.cols["sip6"].to_list() + day.cols["dip6"].to_list()
    keys = np.concatenate([k["sip"], k["dip"]])
    m = {}
    for t, key in zip(txt, keys.tolist()):
        if t:
            assert m.setdefault(t, key) == key
    assert len(set(m.values())) == len(m)


def test_ipv6_results_and_cli_feedback(tmp_path):
    from oni355.cli import ml, oa
    day = _day(6000)
    p = str(tmp_path / "f.csv")
    decoders.write_flow_csv(p, day.cols)
    lp, conf = str(tmp_path / "lp"), str(tmp_path / "none.conf")
    args = ["20160708", "flow", "1.0", "400", "--input", p, "--device", "cpu", "--sweeps", "6", "--lpath", lp,
            "--quiet", "--config", conf]
    assert ml.main(args) == 0
    res = os.path.join(lp, "flow", "20160708", "flow_results.csv")
    rows = list(csv.reader(open(res)))
    h, body = rows[0], rows[1:]
    v6_rows = [i for i, r in enumerate(body) if ":" in r[h.index("sip")]]
    assert v6_rows, "no IPv6 flow among the results"
    # analyst marks an IPv6 result benign; the next run takes it as feedback without error
    assert oa.main(["-d", "20160708", "-t", "flow", "--lpath", lp, "--config", conf]) == 0
    assert oa.main(["score", "-d", "20160708", "-t", "flow", "--lpath", lp, "--config", conf, "--rows",
                    str(v6_rows[0]), "--sev", "3"]) == 0
    assert oa.main(["publish", "-d", "20160708", "-t", "flow", "--lpath", lp, "--config", conf]) == 0
    from oni355.oa.feedback import load_feedback
    fb = load_feedback(os.path.join(lp, "flow_scores.csv"), "flow")
    assert fb is not None and ":" in fb["sip6"].to_list()[0]
    # OA details for IPv6 rows: the event is found in its own edge file, pages link by safe names
    assert oa.main(["details", "-d", "20160708", "-t", "flow", "--lpath", lp, "--config", conf, "-l", "400",
                    "--input", p]) == 0
    import json
    idx = json.load(open(os.path.join(lp, "flow", "20160708", "details", "index.json")))
    r6 = [r for r in idx["rows"] if ":" in r["ip"]]
    assert r6 and all(r["edge_rows"] >= 1 for r in r6) and all(":" not in r["edge"] for r in r6)
    assert oa.main(["report", "-d", "20160708", "-t", "flow", "--lpath", lp, "--config", conf]) == 0
    page = idx["ips"][r6[0]["ip"]]["page"]
    assert ":" not in page and os.path.exists(os.path.join(lp, "flow", "20160708", "ui", page))
    assert ml.main(args) == 0


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    torch.set_num_threads(1)
    from oni355.parallel import comm as pc
    comm = pc.init_from_env("cpu")
    day = _day(5000)
    per = day.n // world
    lo, hi = rank * per, (day.n if rank == world - 1 else (rank + 1) * per)
    cols = {k: (v.slice(lo, hi) if hasattr(v, "offsets") else v[lo:hi]) for k, v in day.cols.items()}
    res = run_flow(cols, K=20, sweeps=4, maxresults=100, device="cpu", comm=comm, row_offset=lo)
    if rank == 0:
        q.put((res.rows, res.scores))
    comm.barrier()
    pc.shutdown()


def test_ipv6_dp_matches_single_process():
    import socket

    import torch.multiprocessing as mp
    one = run_flow(_day(5000).cols, K=20, sweeps=4, maxresults=100, device="cpu")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    rows, scores = q.get(timeout=600)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(one.rows, rows) and np.array_equal(one.scores, scores)


def test_class_e_ipv4_never_shares_a_key_with_ipv6():
    """On a day with IPv6, bogon IPv4 addresses in 240.0.0.0/4 go through the dictionary too: no
    IPv4 document can alias an IPv6 one, and the result text keeps their dotted form."""
    day = _day()
    cols = dict(day.cols)
    sip = np.asarray(cols["sip"]).copy()
    v6 = np.array([bool(t) for t in cols["sip6"].to_list()])
    v4rows = np.nonzero(~v6)[0][:5]
    sip[v4rows] = V6_KEY_BASE + np.arange(5, dtype=np.uint32)  # exactly the first IPv6 keys
    cols["sip"] = sip
    k = with_ipv6_keys(cols)
    keyed_e = k["sip"][v4rows]
    keyed_6 = k["sip"][v6]
    assert not np.isin(keyed_e, keyed_6).any()
    assert np.all(keyed_e >= V6_KEY_BASE)
    txt = k["sip6"].to_list()
    assert [txt[i] for i in v4rows] == [f"240.0.0.{i}" for i in range(5)]
    assert all(txt[i] == day.cols["sip6"].to_list()[i] for i in np.nonzero(v6)[0][:50])


def test_prefetched_device_columns_must_be_ipv6_keyed():
    import torch
    from oni355.pipeline.flow import DEVICE_COLS, to_device
    day = _day(3000)
    with pytest.raises(ValueError, match="IPv6"):
        run_flow(day.cols, K=8, sweeps=2, maxresults=50, device="cpu", device_cols=to_device(day.cols, "cpu"))
    keyed = with_ipv6_keys(day.cols)
    a = run_flow(keyed, K=8, sweeps=2, maxresults=50, device="cpu", device_cols=to_device(keyed, "cpu"))
    b = run_flow(day.cols, K=8, sweeps=2, maxresults=50, device="cpu")
    assert np.array_equal(a.rows, b.rows) and np.array_equal(a.scores, b.scores)
    assert set(DEVICE_COLS) <= set(keyed) and torch is not None
