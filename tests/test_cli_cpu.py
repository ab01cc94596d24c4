"""End-to-end CLI on CPU: oni-ml (flow/dns/proxy, synthetic + raw-file inputs) → oni-oa enrich →
analyst feedback → second oni-ml run (the noise-filter loop)."""
import csv
import os

import numpy as np
import pytest

from oni355 import schema
from oni355.cli import ml, oa


def _rows(path):
    with open(path, newline="") as f:
        r = list(csv.reader(f))
    return r[0], r[1:]


def test_flow_cli_and_feedback_loop(tmp_path):
    lp = str(tmp_path / "lp")
    args = ["20160708", "flow", "1.0", "50", "--synthetic", "6000", "--device", "cpu", "--sweeps", "8",
            "--lpath", lp, "--quiet"]
    assert ml.main(args) == 0
    res = os.path.join(lp, "flow", "20160708", "flow_results.csv")
    header, rows = _rows(res)
    assert header == schema.FLOW_RESULT_COLUMNS and len(rows) == 50
    scores = [float(r[-1]) for r in rows]
    assert scores == sorted(scores)
    assert os.path.exists(os.path.join(lp, "flow", "20160708", "metrics.jsonl"))
    # OA: enrich, analyst marks the top row's source IP benign, publish as feedback
    assert oa.main(["-d", "20160708", "-t", "flow", "--lpath", lp]) == 0
    sc = os.path.join(lp, "flow", "20160708", "flow_scores.csv")
    h2, r2 = _rows(sc)
    assert h2 == schema.FLOW_SCORE_COLUMNS and len(r2) == 50
    top_ip, top_word = rows[0][9], rows[0][-5]
    assert oa.main(["score", "-d", "20160708", "-t", "flow", "--lpath", lp, "--rows", "0", "--sev", "3"]) == 0
    assert oa.main(["publish", "-d", "20160708", "-t", "flow", "--lpath", lp]) == 0
    assert os.path.exists(os.path.join(lp, "flow_scores.csv"))
    # second run with feedback: the benign-marked event must no longer be the most suspicious
    assert ml.main(args) == 0
    _, rows2 = _rows(res)
    first = [(r[9], r[-5]) for r in rows2[:1]]
    assert first != [(top_ip, top_word)]


def test_flow_cli_from_csv_input(tmp_path):
    from oni355.io.decoders import read_flow_csv, write_flow_csv
    from oni355.synth.flow import generate_flows
    day = generate_flows(3000, seed=4)
    p = str(tmp_path / "flows.csv")
    write_flow_csv(p, day.cols)
    cols, bad = read_flow_csv(p)
    assert bad == 0
    for c in ("sip", "dip", "sport", "dport", "ibyt", "ipkt", "trhour", "trminute", "trsec", "proto"):
        assert np.array_equal(np.asarray(cols[c]), np.asarray(day.cols[c])), c
    lp = str(tmp_path / "lp")
    assert ml.main(["20160708", "flow", "--input", p, "--device", "cpu", "--sweeps", "4", "--lpath", lp,
                    "--quiet", "--ldac-out", str(tmp_path / "ldac")]) == 0
    assert os.path.exists(os.path.join(tmp_path, "ldac", "final.beta"))


@pytest.mark.parametrize("source", ["dns", "proxy"])
def test_dns_proxy_cli(tmp_path, source):
    lp = str(tmp_path / "lp")
    inp = []
    if source == "dns":
        from oni355.synth.dns import generate_dns, write_pcap
        day = generate_dns(4000, seed=3)
        write_pcap(day, str(tmp_path / "d.pcap"))
        inp = ["--input", str(tmp_path / "d.pcap"), "--topics", "50"]
    else:
        from oni355.synth.proxy import generate_proxy, write_log
        day = generate_proxy(3000, seed=3)
        write_log(day, str(tmp_path / "p.log"))
        inp = ["--input", str(tmp_path / "p.log")]
    assert ml.main(["20160708", source, "1.0", "40", *inp, "--device", "cpu", "--sweeps", "4", "--lpath", lp,
                    "--quiet"]) == 0
    header, rows = _rows(os.path.join(lp, source, "20160708", f"{source}_results.csv"))
    assert header == schema.result_columns(source) and len(rows) == 40
    assert oa.main(["-d", "20160708", "-t", source, "--lpath", lp]) == 0
    h2, r2 = _rows(os.path.join(lp, source, "20160708", f"{source}_scores.csv"))
    assert h2 == schema.score_columns(source) and len(r2) == 40
    assert oa.main(["score", "-d", "20160708", "-t", source, "--lpath", lp, "--rows", "0,1", "--sev", "3"]) == 0
    assert oa.main(["publish", "-d", "20160708", "-t", source, "--lpath", lp]) == 0
    from oni355.oa.feedback import load_feedback
    fb = load_feedback(os.path.join(lp, f"{source}_scores.csv"), source)
    assert fb is not None and len(next(iter(fb.values()))) == 2
    assert ml.main(["20160708", source, "1.0", "40", *inp, "--device", "cpu", "--sweeps", "4", "--lpath", lp,
                    "--quiet"]) == 0


def test_setup_layout_templates_and_ingest_config(tmp_path):
    """oni-setup (the oni-setup module's role): folders, table definitions, duxbay.conf and
    ingest_conf.json templates that the other entry points consume; idempotent unless --force."""
    import json

    from oni355 import schema
    from oni355.cli import ingest as ingest_cli
    from oni355.cli import setup as setup_cli
    from oni355.config import OniConfig, load_config
    root, lp, st, conf = (str(tmp_path / x) for x in ("store", "data", "stage", "conf"))
    assert setup_cli.main(["--data-root", root, "--lpath", lp, "--stage", st, "--conf-dir", conf]) == 0
    for src in schema.SOURCES:
        t = json.load(open(os.path.join(root, src, "_table.json")))
        assert [c["name"] for c in t["columns"]] == schema.raw_columns(src)
        assert t["results_columns"] == schema.result_columns(src)
        assert os.path.isdir(os.path.join(lp, src)) and os.path.isdir(os.path.join(st, src))
    kinds = {c["name"]: c["kind"] for c in json.load(open(os.path.join(root, "dns", "_table.json")))["columns"]}
    assert kinds["dns_qry_name"] == "string" and kinds["ip_dst"] == "uint32" and kinds["unix_tstamp"] == "int64"
    cfg = load_config(os.path.join(conf, "duxbay.conf"), env={})
    d = OniConfig()
    assert cfg.TOPIC_COUNT == d.TOPIC_COUNT and cfg.DUPFACTOR == d.DUPFACTOR and cfg.SEED == d.SEED
    assert cfg.DATA_ROOT == os.path.abspath(root) and cfg.LPATH == os.path.abspath(lp) and not cfg.extra
    # second run: nothing rewritten; --force rewrites
    r = setup_cli.setup(root, lp, st, conf)
    assert r == {"created_dirs": [], "written": []}
    assert len(setup_cli.setup(root, lp, st, conf, force=True)["written"]) == 5
    # the ingest template drives oni-ingest (empty collector dir → nothing to do, no errors)
    assert ingest_cli.main(["-t", "flow", "--config", os.path.join(conf, "ingest_conf.json"), "--once"]) == 0
