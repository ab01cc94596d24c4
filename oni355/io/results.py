"""ML results CSV writer/reader (``<LPATH>/<source>/<YYYYMMDD>/<source>_results.csv``).

Schema: raw columns in SURVEY.md §2.7 order + derived words + scores, ascending by score
(``oni355.schema.*_RESULT_COLUMNS``; the reference's exact order is unverifiable, §0 F1).
The reference produced it with ``hdfs dfs -getmerge`` of Spark part files ([U-M]).
"""
from __future__ import annotations

import csv
import datetime as _dt
import io
import os

import numpy as np

from .. import schema
from ..ref import spec
from ..store.columnar import StringColumn

_EMPTY = StringColumn.from_list([""])


def ip_str(v) -> str:
    v = int(v) & 0xFFFFFFFF
    return f"{v >> 24}.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}"


def _fmt_time(unix) -> str:
    return _dt.datetime.fromtimestamp(int(unix), tz=_dt.timezone.utc).strftime("%Y-%m-%d %H:%M:%S")


def _fmt(col: str, v) -> str:
    if col in schema.FLOW_IP_COLUMNS:
        return ip_str(v)
    if col in schema.FLOW_TIME_COLUMNS:
        return _fmt_time(v)
    if col in schema.FLOW_FLOAT_COLUMNS:
        return f"{float(v):g}"
    if isinstance(v, (float, np.floating)):
        return repr(float(v))
    return str(v)


def flow_rows(cols: dict, local_rows: np.ndarray, src_words, dst_words, src_scores, dst_scores, scores) -> list[list]:
    """Pure-Python rendering of flow result rows (the specification of :func:`format_flow`)."""
    out = []
    for i, r in enumerate(np.asarray(local_rows, dtype=np.int64)):
        row = [_fmt(c, cols[c][r]) for c in schema.FLOW_COLUMNS]
        row += [spec.flow_word_str(int(src_words[i])), spec.flow_word_str(int(dst_words[i])),
                f"{float(src_scores[i]):.9g}", f"{float(dst_scores[i]):.9g}", f"{float(scores[i]):.9g}"]
        out.append(row)
    return out


_EVENT_IP_COLUMNS = {"ip_src", "ip_dst", "clientip", "serverip"}


def event_rows(source: str, cols: dict, local_rows, words: list[str], scores) -> list[list]:
    """Pure-Python rendering of DNS / proxy result rows (specification of :func:`format_events`)."""
    names = schema.raw_columns(source)
    out = []
    for i, r in enumerate(np.asarray(local_rows, dtype=np.int64)):
        row = []
        for c in names:
            v = cols.get(c)
            if v is None:
                row.append("")
            elif isinstance(v, StringColumn):
                row.append(v[int(r)])
            elif c in _EVENT_IP_COLUMNS:
                row.append(ip_str(v[r]))
            else:
                row.append(str(v[r]))
        if source == "dns" and not row[0]:
            row[0] = _fmt_time(cols["unix_tstamp"][r])
        out.append(row + [words[i], f"{float(scores[i]):.9g}"])
    return out


# ------------------------------------------------------------------------------------------------
# native rendering (csrc/native/csv_format.cpp): typed result columns → CSV text in one C++ pass
# ------------------------------------------------------------------------------------------------
K_INT, K_IP, K_TIME, K_FLOAT, K_SCORE, K_STR, K_FLOWWORD, K_PACKED, K_STR_OR_TIME, K_STR_ROWS = range(10)


class Rendered:
    """CSV text of result rows: ``blob`` (bytes, rows end in '\n') and each row's end offset."""

    def __init__(self, blob: bytes, ends: np.ndarray):
        self.blob, self.ends = blob, np.asarray(ends, dtype=np.int64)

    def __len__(self) -> int:
        return int(self.ends.size)

    def lines(self) -> list[bytes]:
        starts = np.concatenate([[0], self.ends[:-1]]) if self.ends.size else self.ends
        return [self.blob[a:b] for a, b in zip(starts.tolist(), self.ends.tolist())]

    def rows(self) -> list[list[str]]:
        """Parsed back into fields (tests / small consumers)."""
        return list(csv.reader(io.StringIO(self.blob.decode("utf-8", "replace"))))


def _native_format(fields: list[tuple[int, object]], n: int) -> Rendered:
    import ctypes as C

    from ..ops import native
    native.register("oni_csv_format", [C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p,
                                       C.c_int64, C.c_void_p], C.c_int64)
    L = native.lib()
    keep, ptrs, offs, kinds = [], [], [], []
    str_bytes = 0
    for kind, v in fields:
        if kind == K_STR:
            keep += [v.chars if v.chars.size else np.zeros(1, np.uint8), v.offsets]
            ptrs.append(keep[-2].ctypes.data)
            offs.append(v.offsets.ctypes.data)
            str_bytes += int(v.offsets[-1] - v.offsets[0]) if len(v) else 0
        elif kind == K_PACKED:
            words, spec_fields = v
            a = np.ascontiguousarray(words, dtype=np.uint64)
            sp = np.asarray([len(spec_fields)] + [x for sm in spec_fields for x in sm], dtype=np.int64)
            if a.size != n:
                raise ValueError("result column length mismatch")
            keep += [a, sp]
            ptrs.append(a.ctypes.data)
            offs.append(sp.ctypes.data)
        elif kind in (K_STR_OR_TIME, K_STR_ROWS):
            # a whole string column read through a row index (no gather of the strings on the host)
            col, rows, unix = v if kind == K_STR_OR_TIME else (*v, None)
            r = np.ascontiguousarray(rows, dtype=np.int64)
            if r.size != n:
                raise ValueError("result column length mismatch")
            u = np.ascontiguousarray(unix, dtype=np.int64) if unix is not None else None
            ch = col.chars if col.chars.size else np.zeros(1, np.uint8)
            st = (C.c_void_p * 4)(ch.ctypes.data, col.offsets.ctypes.data, r.ctypes.data,
                                  u.ctypes.data if u is not None else None)
            keep += [r, u, ch, col.offsets, st]
            ptrs.append(C.addressof(st))
            offs.append(None)
            str_bytes += int((col.offsets[r + 1] - col.offsets[r]).sum()) if r.size else 0
        else:
            dt = {K_INT: np.int64, K_IP: np.uint32, K_TIME: np.int64, K_FLOAT: np.float64, K_SCORE: np.float32,
                  K_FLOWWORD: np.uint32}[kind]
            a = np.ascontiguousarray(v, dtype=dt)
            if a.size != n:
                raise ValueError("result column length mismatch")
            keep.append(a)
            ptrs.append(a.ctypes.data)
            offs.append(None)
        kinds.append(kind)
    nc = len(kinds)
    kind_a = (C.c_int32 * nc)(*kinds)
    ptr_a = (C.c_void_p * nc)(*ptrs)
    off_a = (C.c_void_p * nc)(*offs)
    ends = np.zeros(max(n, 1), dtype=np.int64)
    cap = max(n * 24 * max(nc, 1) + 2 * str_bytes, 1024)  # typical non-string fields < 24 bytes; retried once if short
    for _ in range(2):
        buf = np.empty(cap, dtype=np.uint8)  # not zeroed: only [0, m) is read back
        m = L.oni_csv_format(n, nc, kind_a, ptr_a, off_a, buf.ctypes.data_as(C.c_char_p), cap, ends.ctypes.data)
        if m < 0:
            raise ValueError("bad result column kind")
        if m <= cap:
            return Rendered(buf[:m].tobytes(), ends[:n].copy())
        cap = int(m)
    raise RuntimeError("csv formatter did not converge")


def _col_field(c: str, v, rows: np.ndarray, ip_cols=(), time_cols=(), float_cols=()):
    if v is None:
        return K_STR, _EMPTY.take(np.zeros(rows.size, np.int64))
    if isinstance(v, StringColumn):
        if type(v) is not StringColumn:  # lazily formatted columns (pcap frame_time): only these rows
            return K_STR, v.take(rows)
        return K_STR_ROWS, (v, rows)
    a = np.asarray(v)[rows]
    if c in ip_cols:
        return K_IP, a.astype(np.int64).astype(np.uint32) if a.dtype != np.uint32 else a
    if c in time_cols:
        return K_TIME, a
    if c in float_cols or a.dtype.kind == "f":
        return K_FLOAT, a
    return K_INT, a


def _ip_text_field(cols: dict, c: str, rows: np.ndarray):
    """sip / dip of result rows as text when the day has IPv6 flows: the IPv6 address where the
    row has one, dotted IPv4 otherwise (only the few result rows are formatted here)."""
    v6 = cols[c + "6"].take(rows).to_list()
    v4 = np.asarray(cols[c])[rows]
    return K_STR, StringColumn.from_list([t if t else ip_str(x) for t, x in zip(v6, v4)])


def format_flow(cols: dict, local_rows, src_words, dst_words, src_scores, dst_scores, scores) -> Rendered:
    rows = np.asarray(local_rows, dtype=np.int64)
    f = [_ip_text_field(cols, c, rows) if (c + "6") in cols else
         _col_field(c, cols[c], rows, schema.FLOW_IP_COLUMNS, schema.FLOW_TIME_COLUMNS, schema.FLOW_FLOAT_COLUMNS)
         for c in schema.FLOW_COLUMNS]
    f += [(K_FLOWWORD, np.asarray(src_words).astype(np.uint32)), (K_FLOWWORD, np.asarray(dst_words).astype(np.uint32)),
          (K_SCORE, src_scores), (K_SCORE, dst_scores), (K_SCORE, scores)]
    return _native_format(f, rows.size)


def format_events(source: str, cols: dict, local_rows, words, scores) -> Rendered:
    """``words``: rendered strings, or ``(packed u64 words, [(shift, mask), ...])`` rendered by the
    native formatter ('_'-joined fields, :func:`word_fields`)."""
    rows = np.asarray(local_rows, dtype=np.int64)
    f = [_col_field(c, cols.get(c), rows, _EVENT_IP_COLUMNS) for c in schema.raw_columns(source)]
    if source == "dns" and rows.size:
        col, r = f[0][1] if f[0][0] == K_STR_ROWS else (f[0][1], np.arange(rows.size))
        if ((col.offsets[r + 1] - col.offsets[r]) == 0).any():
            # frame_time missing: rendered from unix_tstamp where empty
            f[0] = (K_STR_OR_TIME, (col, r, np.asarray(cols["unix_tstamp"])[rows]))
    if isinstance(words, tuple):
        f += [(K_PACKED, words)]
    else:
        f += [(K_STR, StringColumn.from_list(words))]
    f += [(K_SCORE, scores)]
    return _native_format(f, rows.size)


def render_local(source: str, cols: dict, res, row_off: int):
    """(global row ids, Rendered) of the result rows this rank holds (``cols`` is its shard,
    starting at global row ``row_off``), formatted by the native formatter. No collectives."""
    rows_local = res.rows - row_off
    if source == "flow":
        mine = (rows_local >= 0) & (rows_local < len(cols["sip"]))
        rendered = format_flow(cols, rows_local[mine], res.src_words[mine], res.dst_words[mine],
                               res.src_scores[mine], res.dst_scores[mine], res.scores[mine])
    else:
        ncol = len(cols["ip_dst" if source == "dns" else "clientip"])
        mine = (rows_local >= 0) & (rows_local < ncol)
        rendered = format_events(source, cols, rows_local[mine], (res.words[mine], word_fields(source)),
                                 res.scores[mine])
    return res.rows[mine], rendered


def gather_rendered(all_rows: np.ndarray, gids: np.ndarray, rendered: Rendered, comm=None) -> Rendered:
    """Merge every rank's locally rendered rows into the full text in ``all_rows`` order (collective
    X06's payload; every rank returns it). Identity without a process group.

    Each rank's (row ids, line ends, text) travel as one byte tensor through ``Comm.allgather_var``
    (a size exchange + one all-gather on the collective device) -- no pickling."""
    if comm is None or not comm.dist:
        return rendered
    import torch

    g = np.ascontiguousarray(gids, dtype=np.int64)
    e = np.ascontiguousarray(rendered.ends, dtype=np.int64)
    blob = np.frombuffer(rendered.blob, dtype=np.uint8)
    payload = np.concatenate([np.array([g.size, blob.size], np.int64).view(np.uint8), g.view(np.uint8),
                              e.view(np.uint8), blob])
    t = torch.from_numpy(payload)
    if comm.device.type == "cuda":
        t = t.to(comm.device)
    gl, st, en, texts, base = [], [], [], [], 0
    for part in comm.allgather_var(t):
        b = part.cpu().numpy()
        n, nb = (int(x) for x in b[:16].view(np.int64))
        pe = b[16 + 8 * n:16 + 16 * n].view(np.int64)
        gl.append(b[16:16 + 8 * n].view(np.int64))
        st.append(base + np.concatenate([[0], pe[:-1]]) if n else np.zeros(0, np.int64))
        en.append(base + pe)
        texts.append(b[16 + 16 * n:16 + 16 * n + nb].tobytes())
        base += nb
    g_all, s_all, e_all = np.concatenate(gl), np.concatenate(st), np.concatenate(en)
    blob = b"".join(texts)
    o = np.argsort(g_all, kind="stable")
    pos = o[np.searchsorted(g_all[o], np.asarray(all_rows, dtype=np.int64))]
    mv = memoryview(blob)
    out = b"".join(mv[a:b_] for a, b_ in zip(s_all[pos].tolist(), e_all[pos].tolist()))
    ends = np.cumsum(e_all[pos] - s_all[pos]).astype(np.int64)
    return Rendered(out, ends)


def render_result(source: str, cols: dict, res, row_off: int, comm=None) -> Rendered:
    """Result rows of a pipeline run (FlowResult / SingleResult) as CSV text, ascending score.

    Each rank formats the result rows it holds with the native formatter; with a process group the
    formatted rows are gathered and every rank returns the full, globally ordered text."""
    gids, rendered = render_local(source, cols, res, row_off)
    return gather_rendered(res.rows, gids, rendered, comm)


class ResultPipe:
    """Day-pipelined result output: day k's rows are formatted on a worker thread while day k+1
    computes; the cross-rank gather and the write of day k happen on the caller's thread at the
    next :meth:`submit` / :meth:`drain`, so every rank issues its collectives in program order.

    ``write(rendered)`` is called with each day's full text (on every rank; rank 0 usually
    writes). The native formatter runs outside the GIL."""

    def __init__(self, source: str, comm=None, write=None):
        from concurrent.futures import ThreadPoolExecutor

        self.source = source
        self.comm = comm
        self.write = write
        self._pool = ThreadPoolExecutor(1, thread_name_prefix="oni-results")
        self._pending = None  # (future of (gids, Rendered), all result rows)
        # data parallel: the rendered-row gather runs on the worker thread too, over a gloo group
        # of its own (host bytes; never interleaves with the main thread's device collectives)
        self._hcomm = comm.side_group("results") if comm is not None and comm.dist else None

    def submit(self, cols: dict, res, row_off: int, tag=None) -> None:
        """Queue this day's formatting; finishes the previous day first. ``ONI_RESULT_PIPE=0``
        formats and writes inline (no worker thread). ``tag`` (e.g. the day) is passed on to
        ``write(rendered, tag)``."""
        self._finish()
        if os.environ.get("ONI_RESULT_PIPE", "1") == "0":
            from concurrent.futures import Future
            fut = Future()
            fut.set_result(render_local(self.source, cols, res, row_off))
            self._pending = (fut, res.rows, tag)
            self._finish()
            return
        if os.environ.get("ONI_RESULT_GATHER_WORKER", "1") == "1" or self.comm is None or not self.comm.dist:
            # the worker formats, gathers (data parallel: on its own gloo group, days in program
            # order on every rank) AND writes the day
            self._pending = (self._pool.submit(self._local_day, cols, res, row_off, tag), None, "__done__")
            return
        fut = self._pool.submit(render_local, self.source, cols, res, row_off)
        self._pending = (fut, res.rows, tag)

    def _local_day(self, cols: dict, res, row_off: int, tag):
        gids, rendered = render_local(self.source, cols, res, row_off)
        full = gather_rendered(res.rows, gids, rendered, self._hcomm)
        if self.write is not None:
            self.write(full) if tag is None else self.write(full, tag)
        return full

    def _finish(self):
        if self._pending is None:
            return None
        fut, rows, tag = self._pending
        self._pending = None
        if tag == "__done__":
            return fut.result()
        gids, rendered = fut.result()
        full = gather_rendered(rows, gids, rendered, self.comm)
        if self.write is not None:
            self.write(full) if tag is None else self.write(full, tag)
        return full

    def drain(self):
        """Finish the last queued day (its full Rendered text, or None)."""
        return self._finish()

    def close(self) -> None:
        self._finish()
        self._pool.shutdown(wait=True)


def word_fields(source: str) -> list[tuple[int, int]]:
    """(shift, mask) of every field of a DNS / proxy word, in ``word_str`` order."""
    from ..ref import spec as sp
    if source == "dns":
        from ..pipeline import dns as m
        out = [(m.TOP_SHIFT, 3)] + [(s, 15 if fr is sp.DECILES else 7) for _, fr, s in m.BINNED]
        return out + [(s, mk) for _, mk, s in m.RAW]
    from ..pipeline import proxy as m
    fields = {"top": (m.TOP_SHIFT, 3)}
    for name, fr, s in m.BINNED:
        fields[name] = (s, 15 if fr is sp.DECILES else 7)
    for name, mk, s in m.RAW:
        fields[name] = (s, mk)
    return [fields[k] for k in ("top", "time", "method", "ua_freq", "ctype", "uri_ent", "uri_len", "respcode")]


def write_rendered(path: str, header: list[str], rendered: Rendered) -> str:
    """Header + pre-formatted rows (atomic rename)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write((",".join(header) + "\n").encode())
        f.write(rendered.blob)
    os.replace(tmp, path)
    return path


def write_csv(path: str, header: list[str], rows: list[list], with_header: bool = True) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w", newline="") as f:
        w = csv.writer(f, lineterminator="\n")
        if with_header:
            w.writerow(header)
        w.writerows(rows)
    os.replace(tmp, path)
    return path


def read_csv(path: str) -> tuple[list[str], list[list[str]]]:
    with open(path, newline="") as f:
        r = csv.reader(f)
        header = next(r)
        return header, [row for row in r]


def results_path(lpath: str, source: str, date: str) -> str:
    return os.path.join(lpath, source, date, f"{source}_results.csv")


def scores_path(lpath: str, source: str, date: str | None = None) -> str:
    """Feedback file the next ML run reads (reference: ${LPATH}/${DSOURCE}_scores.csv)."""
    if date:
        return os.path.join(lpath, source, date, f"{source}_scores.csv")
    return os.path.join(lpath, f"{source}_scores.csv")
