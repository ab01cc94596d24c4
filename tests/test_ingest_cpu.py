"""Decoders + ingest on CPU: nfcapd (none/LZO/LZ4/bzip2), LZO/LZ4 stream decoding, columnar store,
collector → day partitions → oni-ml from the store."""
import os

import numpy as np
import pytest

from oni355.io import nfcapd
from oni355.store import columnar
from oni355.synth.flow import generate_flows

KEYS = ["sip", "dip", "sport", "dport", "ibyt", "ipkt", "trhour", "trminute", "trsec", "proto", "unix_tstamp"]


@pytest.mark.parametrize("comp", ["none", "lzo", "lz4", "bz2"])
def test_nfcapd_roundtrip(tmp_path, comp):
    day = generate_flows(5000, seed=2)
    p = str(tmp_path / "nfcapd.201607080000")
    nfcapd.write_nfcapd(p, day.cols, comp, per_block=1234)
    if comp == "bz2":
        raw = open(p, "rb").read()
        assert raw.count(b"BZh9") >= 2  # every data block is a real bzip2 stream
    c = nfcapd.read_nfcapd(p)
    for k in KEYS:
        assert np.array_equal(np.asarray(c[k]), np.asarray(day.cols[k])), k


def test_lzo_and_lz4_streams():
    # literal 'abc' + M2 match (dist 3, len 7) + EOF
    assert nfcapd.lzo1x_decompress(bytes([20]) + b"abc" + bytes([200, 0, 17, 0, 0]), 64) == b"abcabcabca"
    # long literal run (zero-extended length) + EOF
    data = bytes(range(256)) * 3
    t = len(data) - 3 - 15
    enc = bytes([0]) + bytes([0]) * (t // 255 if t % 255 else t // 255 - 1) + bytes([t % 255 or 255]) + data + bytes([17, 0, 0])
    assert nfcapd.lzo1x_decompress(enc, 4096) == data
    with pytest.raises(ValueError):
        nfcapd.lzo1x_decompress(bytes([20]) + b"abc" + bytes([200, 9]), 64)  # match before start
    assert nfcapd.lz4_decompress(bytes([0x35]) + b"abc" + bytes([3, 0, 0x10]) + b"x", 64) == b"abcabcabcabcx"
    with pytest.raises(ValueError):
        nfcapd.lz4_decompress(bytes([0x35]) + b"abc" + bytes([9, 0, 0x10]) + b"x", 64)


def test_nfcapd_rejects_garbage(tmp_path):
    p = tmp_path / "junk"
    p.write_bytes(b"\x0c\xa5" + b"\x00" * 400)
    with pytest.raises(OSError):
        nfcapd.read_nfcapd(str(p))


def test_columnar_store(tmp_path):
    from oni355.store.columnar import StringColumn
    cols = {"a": np.arange(10), "s": StringColumn.from_list([f"x{i}" for i in range(10)])}
    columnar.write_day(str(tmp_path), "dns", "20160708", cols)
    columnar.append_part(str(tmp_path), "dns", "20160708", {"a": np.arange(10, 15),
                                                            "s": StringColumn.from_list(["y"] * 5)})
    assert columnar.rows(str(tmp_path), "dns", "20160708") == 15
    d = columnar.read_day(str(tmp_path), "dns", "20160708", row_range=(8, 12))
    assert list(d["a"]) == [8, 9, 10, 11] and d["s"].to_list() == ["x8", "x9", "y", "y"]


def test_collector_to_store_to_ml(tmp_path):
    from oni355.cli import ml
    from oni355.ingest.watch import Collector
    col = tmp_path / "collector"
    col.mkdir()
    day = generate_flows(4000, seed=6)
    half = {k: v[:2000] for k, v in day.cols.items()}
    rest = {k: v[2000:] for k, v in day.cols.items()}
    nfcapd.write_nfcapd(str(col / "nfcapd.201607080000"), half, "lzo")
    nfcapd.write_nfcapd(str(col / "nfcapd.201607080005"), rest, "lz4")
    (col / "ignored.txt").write_text("x")
    root = str(tmp_path / "store")
    c = Collector("flow", str(col), root, workers=2, log=lambda m: None)
    out = c.run_once()
    assert len(out) == 2 and c.stats["rows"] == 4000 and c.stats["errors"] == 0
    assert c.run_once() == []  # idempotent: already ingested
    assert columnar.rows(root, "flow", "20160708") == 4000
    lp = str(tmp_path / "lp")
    assert ml.main(["20160708", "flow", "1.0", "20", "--data-root", root, "--device", "cpu", "--sweeps", "3",
                    "--lpath", lp, "--quiet"]) == 0
    assert os.path.exists(os.path.join(lp, "flow", "20160708", "flow_results.csv"))


@pytest.mark.parametrize("fmt", ["oni", "nfdump"])
def test_oni_nfdump_cli_csv_matches_reader(tmp_path, fmt):
    """oni-nfdump (C++ nfcapd → CSV formatter) output parses back to the same flow columns."""
    import subprocess

    from oni355.io.decoders import read_flow_csv
    exe = os.path.join(os.path.dirname(nfcapd.__file__), "..", "_lib", "bin", "oni-nfdump")
    day = generate_flows(3000, seed=6)
    p1, p2 = str(tmp_path / "nfcapd.a"), str(tmp_path / "nfcapd.b")
    nfcapd.write_nfcapd(p1, {k: v[:1700] for k, v in day.cols.items()}, "lzo", per_block=500)
    nfcapd.write_nfcapd(p2, {k: v[1700:] for k, v in day.cols.items()}, "lz4")
    out = str(tmp_path / "flows.csv")
    r = subprocess.run([exe, "-r", p1, "-r", p2, "-o", fmt, "-w", out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    cols, bad = read_flow_csv(out)
    assert bad == 0
    for k in KEYS:
        assert np.array_equal(np.asarray(cols[k]), np.asarray(day.cols[k])), k
    bad_r = subprocess.run([exe, "-r", str(tmp_path / "missing")], capture_output=True, text=True)
    assert bad_r.returncode == 1 and "cannot open" in bad_r.stderr
