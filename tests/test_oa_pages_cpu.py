"""OA details + analyst pages (oni-oa details / threat / report) and hour partitions of the store.

The reference's OA wrote per-suspicious-row edge/chord/dendrogram TSVs and served suspicious,
threat-investigation, storyboard and ingest-summary views; here: files under <day>/details and
self-contained HTML under <day>/ui, driven from the CLI on a synthetic day."""
import json
import os

import numpy as np
import pytest

from oni355.cli import ml, oa
from oni355.store import columnar

D = "20160708"


def _top_rows(lp, source):
    import csv
    with open(os.path.join(lp, source, D, f"{source}_results.csv"), newline="") as f:
        r = list(csv.reader(f))
    return r[0], r[1:]


def test_flow_details_threat_and_pages(tmp_path):
    from oni355.synth.flow import generate_flows
    root, lp = str(tmp_path / "store"), str(tmp_path / "lp")
    day = generate_flows(6000, seed=9)
    columnar.write_day(root, "flow", D, day.cols)
    conf = str(tmp_path / "none.conf")
    assert ml.main([D, "flow", "1.0", "40", "--data-root", root, "--device", "cpu", "--sweeps", "6", "--lpath", lp,
                    "--quiet", "--config", conf]) == 0
    base = ["-d", D, "-t", "flow", "--lpath", lp, "--config", conf]
    assert oa.main(base) == 0
    assert oa.main(["details", *base, "-l", "10", "--data-root", root]) == 0
    det = os.path.join(lp, "flow", D, "details")
    idx = json.load(open(os.path.join(det, "index.json")))
    header, rows = _top_rows(lp, "flow")
    assert len(idx["rows"]) == 10
    for ent, r in zip(idx["rows"], rows):
        sip, dip, hh = r[header.index("sip")], r[header.index("dip")], int(r[header.index("trhour")])
        assert ent["edge"] == f"edge-{sip}-{dip}-{hh:02d}.tsv"  # IPv4 names are already file-safe
        lines = open(os.path.join(det, ent["edge"])).read().splitlines()
        assert ent["edge_rows"] >= 1 and len(lines) == ent["edge_rows"] + 1  # the event itself is in its edge
        assert os.path.exists(os.path.join(det, idx["ips"][sip]["chord"])) and os.path.exists(os.path.join(det, idx["ips"][sip]["timeline"]))
    summ = open(os.path.join(det, "ingest_summary.tsv")).read().splitlines()
    assert sum(int(x.split("\t")[1]) for x in summ[1:]) == 6000
    ip = idx["rows"][0]["ip"]
    assert oa.main(["threat", *base, "--ip", ip, "--title", "Beaconing", "--comment", "odd hour <b>exfil</b>"]) == 0
    assert oa.main(["report", *base]) == 0
    ui = os.path.join(lp, "flow", D, "ui")
    for pg in ("suspicious.html", "storyboard.html", "ingest_summary.html", f"threat-{ip}.html"):
        assert os.path.exists(os.path.join(ui, pg)), pg
    th = open(os.path.join(ui, f"threat-{ip}.html")).read()
    assert "<svg" in th and "Beaconing" in th and "&lt;b&gt;exfil&lt;/b&gt;" in th  # escaped analyst text
    assert f'href="threat-{ip}.html"' in open(os.path.join(ui, "suspicious.html")).read()


@pytest.mark.parametrize("source", ["dns", "proxy"])
def test_dns_proxy_details_from_raw_files(tmp_path, source):
    lp = str(tmp_path / "lp")
    conf = str(tmp_path / "none.conf")
    if source == "dns":
        from oni355.synth.dns import generate_dns, write_pcap
        day = generate_dns(3000, seed=4)
        inp = str(tmp_path / "d.pcap")
        write_pcap(day, inp)
        extra = ["--topics", "50"]
    else:
        from oni355.synth.proxy import generate_proxy, write_log
        day = generate_proxy(3000, seed=4)
        inp = str(tmp_path / "p.log")
        write_log(day, inp)
        extra = []
    assert ml.main([D, source, "1.0", "30", "--input", inp, *extra, "--device", "cpu", "--sweeps", "4", "--lpath", lp,
                    "--quiet", "--config", conf]) == 0
    base = ["-d", D, "-t", source, "--lpath", lp, "--config", conf]
    assert oa.main(base) == 0
    assert oa.main(["details", *base, "-l", "5", "--input", inp]) == 0
    det = os.path.join(lp, source, D, "details")
    idx = json.load(open(os.path.join(det, "index.json")))
    assert len(idx["rows"]) == 5 and all(r["edge_rows"] >= 1 for r in idx["rows"])
    if source == "dns":
        assert all(os.path.exists(os.path.join(det, e["dendro"])) for e in idx["ips"].values())
    assert oa.main(["report", *base]) == 0
    assert os.path.exists(os.path.join(lp, source, D, "ui", "suspicious.html"))


def test_hour_partitions_ingest_and_reads(tmp_path):
    from oni355.ingest.watch import store_rows
    from oni355.oa import details
    from oni355.synth.flow import generate_flows
    day = generate_flows(5000, seed=2)
    root = str(tmp_path / "store")
    got = store_rows(root, "flow", day.cols)
    assert got == {D: 5000}
    hrs = columnar.hours(root, "flow", D)
    want = np.bincount(np.asarray(day.cols["trhour"]), minlength=24)
    assert hrs == [h for h in range(24) if want[h]]
    assert columnar.rows(root, "flow", D) == 5000
    for h in hrs[:3]:
        c = columnar.read_day(root, "flow", D, hours=[h])
        assert len(c["sip"]) == want[h] and np.all(np.asarray(c["trhour"]) == h)
    assert details.ingest_summary(root, "flow", D) == [(h, int(want[h])) for h in range(24)]


def test_proxy_day_hour_vectorised_matches_python():
    import datetime as dt

    from oni355.ingest.watch import _row_day_hour
    from oni355.store.columnar import StringColumn
    dates = ["2016-07-08", "1999-12-31", "2024-02-29", "", "2016-01-01"]
    times = ["13:05:00", "00:00:01", "23:59:59", "", "07:30:00"]
    d, h = _row_day_hour("proxy", {"p_date": StringColumn.from_list(dates), "p_time": StringColumn.from_list(times)})
    ref = [(dt.date.fromisoformat(x) - dt.date(1970, 1, 1)).days if x else 0 for x in dates]
    assert d.tolist() == ref and h.tolist() == [13, 0, 23, 0, 7]
