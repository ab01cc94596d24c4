"""Native result formatter (csrc/native/csv_format.cpp) == the pure-Python row specification."""
import csv
import io

import numpy as np

from oni355 import schema
from oni355.io import results as rio
from oni355.store.columnar import StringColumn
from oni355.synth.dns import generate_dns
from oni355.synth.flow import generate_flows
from oni355.synth.proxy import generate_proxy


def _parse(rendered):
    return list(csv.reader(io.StringIO(rendered.blob.decode())))


def test_flow_rows_native_equals_python():
    day = generate_flows(3000, seed=4)
    r = np.random.default_rng(0)
    rows = r.choice(3000, 257, replace=False)
    sw = r.integers(0, 1 << 29, 257).astype(np.uint32)
    sw[:5] = [65536 << 11, (65537 << 11) | (1 << 28), 53 << 11, 0, (1 << 28) | (80 << 11) | 0x7F]
    dw = r.integers(0, 1 << 29, 257).astype(np.uint32)
    s1, s2 = r.random(257).astype(np.float32) * 1e-3, r.random(257).astype(np.float32)
    sc = np.minimum(s1, s2)
    sc[0], sc[1] = np.float32(1e-30), np.float32(0.0)
    want = rio.flow_rows(day.cols, rows, sw, dw, s1, s2, sc)
    got = rio.format_flow(day.cols, rows, sw, dw, s1, s2, sc)
    assert len(got) == 257 and _parse(got) == want
    assert got.lines()[3] == got.blob[got.ends[2]:got.ends[3]]


def test_event_rows_native_equals_python_with_quoting():
    for source, day in (("dns", generate_dns(2000, seed=3)), ("proxy", generate_proxy(2000, seed=3))):
        cols = dict(day.cols)
        if source == "proxy":
            ua = cols["useragent"].to_list()
            ua[0], ua[1], ua[2] = 'Mozilla/5.0 (X11, "quoted")', "a,b", "line\nbreak"
            cols["useragent"] = StringColumn.from_list(ua)
        rows = np.arange(0, 2000, 7)
        words = [f"{i}_1_2" for i in range(rows.size)]
        sc = np.linspace(1e-9, 1e-3, rows.size).astype(np.float32)
        want = rio.event_rows(source, cols, rows, words, sc)
        got = rio.format_events(source, cols, rows, words, sc)
        assert _parse(got) == want, source


def test_string_column_take():
    c = StringColumn.from_list(["ab", "", "cde", "f"])
    t = c.take([2, 1, 0, 2])
    assert t.to_list() == ["cde", "", "ab", "cde"]
    assert c.take([]).to_list() == []


def test_write_rendered_roundtrip(tmp_path):
    day = generate_flows(500, seed=1)
    rend = rio.format_flow(day.cols, np.arange(10), np.zeros(10, np.uint32), np.zeros(10, np.uint32),
                           np.ones(10, np.float32), np.ones(10, np.float32), np.ones(10, np.float32))
    p = rio.write_rendered(str(tmp_path / "x" / "flow_results.csv"), schema.FLOW_RESULT_COLUMNS, rend)
    header, body = rio.read_csv(p)
    assert header == schema.FLOW_RESULT_COLUMNS and len(body) == 10


def test_native_event_rendering_many_rows_matches_spec():
    """Several formatter row blocks (parallel path), string columns read through the row index,
    packed DNS / proxy words rendered natively, empty frame_time falling back to unix_tstamp."""
    import numpy as np

    from oni355.io import results as rio
    from oni355.pipeline.dns import word_str as dws
    from oni355.pipeline.proxy import word_str as pws
    from oni355.synth.dns import generate_dns
    from oni355.synth.proxy import generate_proxy
    rng = np.random.default_rng(5)
    for src, day, ws in (("dns", generate_dns(20_000, seed=2), dws), ("proxy", generate_proxy(20_000, seed=2), pws)):
        rows = rng.permutation(20_000)[:2500]  # score order: not ascending rows
        w = rng.integers(0, 2**40, rows.size).astype(np.uint64)
        sc = rng.random(rows.size).astype(np.float32)
        got = rio.format_events(src, day.cols, rows, (w, rio.word_fields(src)), sc)
        assert got.rows() == rio.event_rows(src, day.cols, rows, [ws(x) for x in w], sc)
        assert len(got) == rows.size and got.ends[-1] == len(got.blob)


def test_result_pipe_writes_each_day_like_render_result():
    """ResultPipe (format on a worker thread, gather + write at the next submit / drain) emits
    exactly render_result's text for every day, in day order."""
    from types import SimpleNamespace

    day = generate_flows(2000, seed=6)
    r = np.random.default_rng(1)
    days = []
    for k in range(3):
        n = 50 + 10 * k
        rows = r.choice(2000, n, replace=False).astype(np.int64)
        s = np.sort(r.random(n).astype(np.float32))
        days.append(SimpleNamespace(rows=rows, scores=s, src_scores=s, dst_scores=s + 1,
                                    src_words=r.integers(0, 1 << 29, n).astype(np.uint32),
                                    dst_words=r.integers(0, 1 << 29, n).astype(np.uint32)))
    out = []
    pipe = rio.ResultPipe("flow", None, write=out.append)
    for res in days:
        pipe.submit(day.cols, res, 0)
    assert len(out) == 2
    assert pipe.drain() is not None and pipe.drain() is None
    pipe.close()
    assert [o.blob for o in out] == [rio.render_result("flow", day.cols, res, 0).blob for res in days]


def test_result_pipe_inline_mode(monkeypatch):
    """ONI_RESULT_PIPE=0 formats and writes each day at its own submit (no worker thread)."""
    from types import SimpleNamespace

    monkeypatch.setenv("ONI_RESULT_PIPE", "0")
    day = generate_flows(1000, seed=2)
    rows = np.arange(0, 40, dtype=np.int64)
    s = np.linspace(0, 1, 40).astype(np.float32)
    res = SimpleNamespace(rows=rows, scores=s, src_scores=s, dst_scores=s,
                          src_words=np.zeros(40, np.uint32), dst_words=np.ones(40, np.uint32))
    out = []
    pipe = rio.ResultPipe("flow", None, write=out.append)
    pipe.submit(day.cols, res, 0)
    assert len(out) == 1 and out[0].blob == rio.render_result("flow", day.cols, res, 0).blob
    assert pipe.drain() is None
    pipe.close()
