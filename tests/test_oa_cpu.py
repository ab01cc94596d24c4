"""Operational-analytics layer: range-table enrichment (geo, network
context), reputation plugins, IANA names, detail queries, scores-file enrichment and the analyst
severity / feedback round trip. All CPU, hand-built inputs (the reference shipped no tests, §4.1)."""
from __future__ import annotations

import csv
import os

import numpy as np
import pytest

from oni355 import schema
from oni355.io import results as rio
from oni355.oa import details, enrich, feedback, iana, reputation


def _ipi(s: str) -> int:
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


# ---- C28 / C29: range tables --------------------------------------------------------------------
def test_range_table_geo_and_cidr(tmp_path):
    p = tmp_path / "iploc.csv"
    p.write_text("# start,end,location\n"
                 f"{_ipi('1.0.0.0')},{_ipi('1.0.0.255')},AU,Queensland,Brisbane\n"
                 "8.8.8.0,8.8.8.255,US,California\n"
                 "header,row,ignored\n")
    t = enrich.RangeTable.from_csv(str(p))
    got = t.lookup([_ipi("1.0.0.7"), _ipi("8.8.8.8"), _ipi("8.8.9.1"), _ipi("0.255.255.255"), _ipi("1.0.0.255")])
    assert got == ["AU,Queensland,Brisbane", "US,California", "", "", "AU,Queensland,Brisbane"]

    nc = tmp_path / "networkcontext.csv"
    nc.write_text("10.1.0.0/16,datacenter\n192.168.1.0/24,lab\n")
    t2 = enrich.RangeTable.from_csv(str(nc))
    assert t2.lookup([_ipi("10.1.200.3"), _ipi("10.2.0.1"), _ipi("192.168.1.255")]) == ["datacenter", "", "lab"]

    d = enrich.default_context()
    assert d.lookup([_ipi("10.9.9.9"), _ipi("172.31.0.1"), _ipi("172.32.0.1"), _ipi("8.8.8.8")]) == \
        ["internal", "internal", "", ""]
    assert enrich.RangeTable([], [], []).lookup([1, 2]) == ["", ""]


# ---- C30: reputation plugins --------------------------------------------------------------------
def test_csv_reputation_exact_and_suffix(tmp_path):
    p = tmp_path / "rep.csv"
    p.write_text("# indicator,verdict\n6.6.6.6,malicious\nevil.example.com,high\nbad.org\n")
    svc = reputation.CsvReputation(str(p))
    got = svc.check(["6.6.6.6", "a.b.evil.example.com", "http://x.bad.org/path?q=1", "good.org", "EVIL.example.com"])
    assert got == {"6.6.6.6": "malicious", "a.b.evil.example.com": "high", "http://x.bad.org/path?q=1": "listed",
                   "good.org": "", "EVIL.example.com": "high"}
    svcs = reputation.load_services(f"csv:{p}")
    assert len(svcs) == 1 and svcs[0].name == "csv"
    assert reputation.load_services(None) == [] and reputation.load_services(" ") == []
    # networked services are registered but refuse to run without egress
    cfg = tmp_path / "gti.json"
    cfg.write_text('{"server": "x"}')
    with pytest.raises(RuntimeError):
        reputation.load_services(f"gti:{cfg}")
    with pytest.raises(FileNotFoundError):
        reputation.FbThreatExchange(str(tmp_path / "missing.json"))
    # multi-service join format
    assert enrich._rep([svc, svc], ["6.6.6.6", "1.1.1.1"]) == ["csv:malicious::csv:malicious", ""]


# ---- C31: IANA names ----------------------------------------------------------------------------
def test_iana_tables():
    assert iana.dns_type(1) == "A" and iana.dns_type(28) == "AAAA" and iana.dns_type(65) == "HTTPS"
    assert iana.dns_class(1) == "IN" and iana.dns_rcode(3) == "NXDomain"
    assert iana.http_status(404) == "Not Found" and iana.http_status(599) == "599"
    assert iana.dns_type(9999) == "9999"


# ---- C32: detail queries ------------------------------------------------------------------------
def _flow_cols():
    rng = np.random.default_rng(3)
    n = 200
    a, b, c = _ipi("10.0.0.1"), _ipi("10.0.0.2"), _ipi("10.0.0.3")
    sip = rng.choice([a, b, c], n).astype(np.uint32)
    dip = rng.choice([a, b, c], n).astype(np.uint32)
    return {
        "sip": sip, "dip": dip, "sport": rng.integers(1, 65535, n), "dport": rng.integers(1, 1024, n),
        "proto": np.full(n, 6), "ipkt": rng.integers(1, 100, n), "ibyt": rng.integers(40, 10_000, n),
        "opkt": rng.integers(1, 10, n), "obyt": rng.integers(40, 500, n), "tdur": rng.random(n),
        "trhour": rng.integers(0, 24, n), "unix_tstamp": 1467936000 + rng.integers(0, 86400, n),
    }, (a, b, c)


def test_edge_chord_timeline():
    cols, (a, b, c) = _flow_cols()
    m = ((cols["sip"] == a) & (cols["dip"] == b)) | ((cols["sip"] == b) & (cols["dip"] == a))
    e = details.edge_details(cols, "10.0.0.1", "10.0.0.2")
    assert len(e) == int(m.sum())
    assert all({r["sip"], r["dip"]} == {"10.0.0.1", "10.0.0.2"} for r in e)
    h = int(cols["trhour"][np.nonzero(m)[0][0]])
    eh = details.edge_details(cols, a, b, hour=h, limit=3)
    assert 1 <= len(eh) <= 3
    # chord: bytes per peer match a direct sum (self-loops count the IP as its own peer)
    ch = details.chord(cols, "10.0.0.3")
    assert ch and all(x[0] == "10.0.0.3" for x in ch)
    tot = {x[1]: x[2] for x in ch}
    for peer in (a, b, c):
        mm = ((cols["sip"] == c) & (cols["dip"] == peer)) | ((cols["dip"] == c) & (cols["sip"] == peer))
        if peer == c:
            mm = (cols["sip"] == c) & (cols["dip"] == c)
        want = int(cols["ibyt"][mm].sum())
        assert tot.get(rio.ip_str(peer), 0) == want
    assert [x[2] for x in ch] == sorted((x[2] for x in ch), reverse=True)
    assert details.chord(cols, "1.2.3.4") == []
    tl = details.timeline(cols, "10.0.0.1", bucket_s=3600)
    assert sum(n for _, n in tl) == int(((cols["sip"] == a) | (cols["dip"] == a)).sum())
    assert all(t % 3600 == 0 for t, _ in tl)


def test_write_tsv(tmp_path):
    p = details.write_tsv(str(tmp_path / "sub" / "edge-x.tsv"), ["a", "b"], [{"a": 1, "b": 2}, (3, 4)])
    rows = list(csv.reader(open(p), delimiter="\t"))
    assert rows == [["a", "b"], ["1", "2"], ["3", "4"]]


# ---- C27 + C33: enrichment → scores CSV → analyst severity → feedback columns ---------------------
def _flow_results(path):
    rows = []
    for i, (s, d) in enumerate([("10.0.0.5", "8.8.8.8"), ("172.16.4.4", "10.0.0.5"), ("1.2.3.4", "5.6.7.8")]):
        rec = {c: "0" for c in schema.FLOW_COLUMNS}
        rec.update({"treceived": f"2016-07-08 0{i}:1{i}:2{i}", "sip": s, "dip": d, "sport": str(1000 + i),
                    "dport": "80", "proto": "TCP", "ipkt": str(3 + i), "ibyt": str(300 + i), "tdur": "0.5"})
        row = [rec[c] for c in schema.FLOW_COLUMNS] + ["80_1_2_3", "-1_80_1_2_3", "1e-5", "2e-5", "1e-5"]
        rows.append(row)
    rio.write_csv(path, schema.FLOW_RESULT_COLUMNS, rows)


def test_flow_enrich_severity_feedback(tmp_path):
    res = str(tmp_path / "flow_results.csv")
    _flow_results(res)
    geo = enrich.RangeTable([_ipi("8.8.8.0")], [_ipi("8.8.8.255")], ["US"])
    rep_p = tmp_path / "rep.csv"
    rep_p.write_text("1.2.3.4,suspicious\n")
    out = str(tmp_path / "flow_scores.csv")
    n = enrich.enrich("flow", res, out, geo=geo, reputation=reputation.load_services(f"csv:{rep_p}"))
    assert n == 3
    header, rows = rio.read_csv(out)
    assert header == schema.FLOW_SCORE_COLUMNS
    ix = {h: i for i, h in enumerate(header)}
    assert [r[ix["sev"]] for r in rows] == ["0", "0", "0"]
    assert rows[0][ix["dstGeo"]] == "US" and rows[0][ix["srcGeo"]] == ""
    assert rows[0][ix["srcDomain"]] == "internal" and rows[1][ix["srcDomain"]] == "internal"
    assert rows[2][ix["srcIP_rep"]] == "csv:suspicious" and rows[2][ix["dstIP_rep"]] == ""
    # limit
    assert enrich.enrich("flow", res, str(tmp_path / "lim.csv"), limit=1) == 1

    # nothing is benign yet → no feedback
    assert feedback.load_feedback(out, "flow") is None
    assert feedback.set_severity(out, schema.SEV_LOW, ip="10.0.0.5") == 2
    assert feedback.set_severity(out, schema.SEV_LOW, ip="10.0.0.5") == 0  # idempotent
    assert feedback.set_severity(out, schema.SEV_HIGH, rows=[2]) == 1
    fb = feedback.load_feedback(out, "flow")
    assert fb is not None and fb["sip"].size == 2
    assert fb["sip"].tolist() == [_ipi("10.0.0.5"), _ipi("172.16.4.4")]
    assert fb["trhour"].tolist() == [0, 1] and fb["trminute"].tolist() == [10, 11] and fb["trsec"].tolist() == [20, 21]
    assert fb["dport"].tolist() == [80, 80] and fb["ibyt"].tolist() == [300, 301]
    hi = feedback.load_feedback(out, "flow", sev=schema.SEV_HIGH)
    assert hi["sip"].tolist() == [_ipi("1.2.3.4")]
    assert not os.path.exists(out + ".tmp")


def test_dns_and_proxy_enrich(tmp_path):
    dres = str(tmp_path / "dns_results.csv")
    rec = {"frame_time": "Jul  8 2016 10:00:00", "unix_tstamp": "1467972000", "frame_len": "120",
           "ip_src": "10.0.0.53", "ip_dst": "10.0.0.9", "dns_qry_name": "a1b2c3.evil.co.uk", "dns_qry_type": "16",
           "dns_qry_class": "1", "dns_qry_rcode": "3", "dns_a": ""}
    rio.write_csv(dres, schema.DNS_RESULT_COLUMNS, [[rec[c] for c in schema.DNS_COLUMNS] + ["0_1_2_3_4_5_16_3", "1e-6"]])
    dout = str(tmp_path / "dns_scores.csv")
    assert enrich.enrich("dns", dres, dout) == 1
    header, rows = rio.read_csv(dout)
    assert header == schema.DNS_SCORE_COLUMNS
    r = dict(zip(header, rows[0]))
    assert r["domain"] == "evil.co.uk" and r["subdomain"] == "a1b2c3" and r["subdomain_length"] == "6"
    assert r["dns_qry_type_name"] == "TXT" and r["dns_qry_rcode_name"] == "NXDomain" and r["dns_qry_class_name"] == "IN"
    assert r["network_context"] == "internal" and r["top_domain"] == "0"
    assert abs(float(r["subdomain_entropy"]) - np.log2(6)) < 1e-5
    feedback.set_severity(dout, schema.SEV_LOW, ip="10.0.0.9")
    fb = feedback.load_feedback(dout, "dns")
    assert fb["ip_dst"].tolist() == [_ipi("10.0.0.9")] and fb["dns_qry_type"].tolist() == [16]
    assert fb["dns_qry_name"].to_list() == ["a1b2c3.evil.co.uk"]

    pres = str(tmp_path / "proxy_results.csv")
    prec = {c: "" for c in schema.PROXY_COLUMNS}
    prec.update({"p_date": "2016-07-08", "p_time": "13:14:15", "clientip": "192.168.0.7", "host": "x.bad.org",
                 "reqmethod": "GET", "useragent": "curl/7", "respcode": "404", "fulluri": "http://x.bad.org/a"})
    rio.write_csv(pres, schema.PROXY_RESULT_COLUMNS, [[prec[c] for c in schema.PROXY_COLUMNS] + ["w", "3e-7"]])
    rep_p = tmp_path / "rep.csv"
    rep_p.write_text("bad.org,phishing\n")
    pout = str(tmp_path / "proxy_scores.csv")
    assert enrich.enrich("proxy", pres, pout, reputation=reputation.load_services(f"csv:{rep_p}")) == 1
    header, rows = rio.read_csv(pout)
    assert header == schema.PROXY_SCORE_COLUMNS
    r = dict(zip(header, rows[0]))
    assert r["respcode_name"] == "Not Found" and r["uri_rep"] == "csv:phishing" and r["network_context"] == "internal"
    feedback.set_severity(pout, schema.SEV_LOW, rows=[0])
    fb = feedback.load_feedback(pout, "proxy")
    assert fb["clientip"].tolist() == [_ipi("192.168.0.7")] and fb["respcode"].tolist() == [404]
    assert fb["p_time"].to_list() == ["13:14:15"]
