"""Telemetry decoders (Python side of ``liboni_native``): nfdump/ONI flow CSV, pcap DNS, proxy logs.

* :func:`read_flow_csv`  -- oni-nfdump CSV (27 ONI fields) or stock ``nfdump -o csv`` (header-driven)
* :func:`read_pcap_dns`  -- DNS responses from pcap/pcapng (the tshark fields of SURVEY.md §2.2 C02)
* :func:`write_pcap_dns` -- our own pcap writer (synthetic DNS days)
* :func:`read_proxy_log` -- Bluecoat-style access logs (C03)
"""
from __future__ import annotations

import ctypes as C
import os
import datetime as _dt

import numpy as np

from .. import schema
from ..ops import native
from ..store.columnar import StringColumn

vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int

native.register("oni_csv_count_rows", [C.c_char_p, i32, i32], i64)
native.register("oni_csv_parse", [C.c_char_p, i32, i32, vp, vp, i64, vp, C.c_char, i32], i64)
native.register("oni_pcap_dns_open", [C.c_char_p, i32], vp)
native.register("oni_pcap_dns_sizes", [vp, vp, vp, vp, vp], i32)
native.register("oni_pcap_dns_fetch", [vp] + [vp] * 11, i32)
native.register("oni_pcap_dns_free", [vp], None)
native.register("oni_pcap_dns_stats", [vp, vp], i32)
native.register("oni_pcap_dns_write", [C.c_char_p, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32], i64)

native.register("oni_ip_parse_spans", [vp, vp, i64, vp, vp, vp], i64)
native.register("oni_ipv6_text", [vp, i64, vp, i64, vp, vp], i32)

SKIP, I64, F64, IPV4, PROTO, FLAGS, TIME, STR = range(8)
IPANY = -1  # Python-side kind: parsed as text spans, then IPv4 -> u32 column, IPv6 -> "<col>6" text column


def ipv6_text(addrs: np.ndarray, is_v6: np.ndarray, stride: int = 16) -> StringColumn:
    """RFC 5952 text of the 16-byte addresses of the IPv6 rows (empty strings elsewhere)."""
    a = np.ascontiguousarray(addrs, dtype=np.uint8)
    f = np.ascontiguousarray(is_v6, dtype=np.uint8)
    n = f.size
    off = np.zeros(n + 1, np.int64)
    L = native.lib()
    if L.oni_ipv6_text(a.ctypes.data, stride, f.ctypes.data, n, off.ctypes.data, None):
        raise ValueError("bad IPv6 address")
    buf = np.zeros(max(int(off[-1]), 1), np.uint8)
    L.oni_ipv6_text(a.ctypes.data, stride, f.ctypes.data, n, off.ctypes.data, buf.ctypes.data)
    return StringColumn(off, buf[: off[-1]])


def parse_ip_spans(buf: np.ndarray, spans: np.ndarray):
    """(u32 IPv4 [n], IPv6 16-byte rows [n,16], kind [n]: 0 v4, 1 v6, 2 unparsable) of text spans."""
    sp = np.ascontiguousarray(spans, dtype=np.int64).reshape(-1, 2)
    n = sp.shape[0]
    b = np.ascontiguousarray(buf, dtype=np.uint8) if len(buf) else np.zeros(1, np.uint8)
    v4 = np.zeros(n, np.uint32)
    v6 = np.zeros((n, 16), np.uint8)
    kind = np.zeros(n, np.uint8)
    native.lib().oni_ip_parse_spans(b.ctypes.data, sp.ctypes.data, n, v4.ctypes.data, v6.ctypes.data,
                                    kind.ctypes.data)
    return v4, v6, kind


def attach_ipv6(cols: dict, name: str, v6: np.ndarray, kind: np.ndarray) -> None:
    """Add the ``<name>6`` text column when any row is IPv6 (sip6 / dip6)."""
    if np.any(kind == 1):
        cols[name + "6"] = ipv6_text(v6, (kind == 1).astype(np.uint8))

# ONI flow CSV (oni-nfdump output order == Hive flow schema minus unix_tstamp)
_ONI_FLOW_FIELDS = [
    ("treceived", TIME), ("tryear", I64), ("trmonth", I64), ("trday", I64), ("trhour", I64), ("trminute", I64),
    ("trsec", I64), ("tdur", F64), ("sip", IPANY), ("dip", IPANY), ("sport", I64), ("dport", I64), ("proto", PROTO),
    ("flag", FLAGS), ("fwd", I64), ("stos", I64), ("ipkt", I64), ("ibyt", I64), ("opkt", I64), ("obyt", I64),
    ("input", I64), ("output", I64), ("sas", I64), ("das", I64), ("dtos", I64), ("dir", I64), ("rip", IPV4),
]
# stock nfdump -o csv header names -> (our column, kind)
_NFDUMP_MAP = {
    "ts": ("treceived", TIME), "td": ("tdur", F64), "sa": ("sip", IPANY), "da": ("dip", IPANY), "sp": ("sport", I64),
    "dp": ("dport", I64), "pr": ("proto", PROTO), "flg": ("flag", FLAGS), "fwd": ("fwd", I64), "stos": ("stos", I64),
    "ipkt": ("ipkt", I64), "ibyt": ("ibyt", I64), "opkt": ("opkt", I64), "obyt": ("obyt", I64), "in": ("input", I64),
    "out": ("output", I64), "sas": ("sas", I64), "das": ("das", I64), "dtos": ("dtos", I64), "dir": ("dir", I64),
    "ra": ("rip", IPV4),
}
FLOW_V6_COLUMNS = ("sip6", "dip6")
_INT32_COLS = {"tryear", "trmonth", "trday", "trhour", "trminute", "trsec", "sport", "dport", "proto", "flag", "fwd",
               "stos", "input", "output", "sas", "das", "dtos", "dir"}


def _parse(path: str, fields: list[tuple[str | None, int]], skip_header: bool, sep: str = ",", threads: int = 0):
    L = native.lib()
    bpath = path.encode()
    n = L.oni_csv_count_rows(bpath, int(skip_header), threads)
    if n < 0:
        raise OSError(f"cannot read {path}")
    outs, arrs = [], {}
    kinds = np.array([k for _, k in fields], dtype=np.int32)
    for name, k in fields:
        if name is None or k == SKIP:
            outs.append(None)
            continue
        dt = {I64: np.int64, F64: np.float64, IPV4: np.uint32, PROTO: np.int32, FLAGS: np.int32, TIME: np.int64,
              STR: np.int64}.get(k)
        a = np.zeros(n * 2 if k == STR else n, dtype=np.int64 if k == STR else dt)
        arrs[name] = a
        outs.append(a.ctypes.data)
    optr = (C.c_void_p * len(outs))(*outs)
    valid = np.zeros(n, dtype=np.uint8)
    got = L.oni_csv_parse(bpath, int(skip_header), len(fields), kinds.ctypes.data, optr, n, valid.ctypes.data,
                          sep.encode(), threads)
    if got < 0:
        raise OSError(f"parse failed for {path} ({got})")
    m = valid.astype(bool)
    return {k: v[m] if v.size == n else v.reshape(n, 2)[m] for k, v in arrs.items()}, int((~m).sum())


def read_flow_csv(path: str, threads: int = 0) -> tuple[dict, int]:
    """Decode a flow CSV into flow-schema columns. Returns (cols, n_bad_rows)."""
    with open(path, "rb") as f:
        first = f.readline().decode("utf-8", "replace").strip()
    heads = [h.strip().lower() for h in first.split(",")]
    has_header = not any(ch.isdigit() for ch in heads[0][:4]) if heads else False
    if has_header and heads[0] in ("ts", "te"):
        fields = [(_NFDUMP_MAP.get(h, (None, SKIP))) for h in heads]
    elif has_header and heads[0] in ("treceived", "tr"):
        fields = list(_ONI_FLOW_FIELDS)
    else:
        fields = list(_ONI_FLOW_FIELDS)
    anyip = [name for name, k in fields if k == IPANY]
    cols, bad = _parse(path, [(nm, STR if k == IPANY else k) for nm, k in fields], has_header, threads=threads)
    if anyip:
        buf = np.memmap(path, dtype=np.uint8, mode="r") if os.path.getsize(path) else np.zeros(0, np.uint8)
        keep = None
        for name in anyip:
            v4, v6, kind = parse_ip_spans(buf, cols[name])
            cols[name] = v4
            attach_ipv6(cols, name, v6, kind)
            ok = kind != 2
            keep = ok if keep is None else keep & ok
        if keep is not None and not keep.all():  # unparsable address text: a bad row, as before
            bad += int((~keep).sum())
            idx = np.nonzero(keep)[0]
            cols = {k: (v.take(idx) if isinstance(v, StringColumn) else v[idx]) for k, v in cols.items()}
    return finish_flow_cols(cols), bad


def finish_flow_cols(cols: dict) -> dict:
    n = len(next(iter(cols.values()))) if cols else 0
    t = cols.get("treceived", np.zeros(n, np.int64))
    cols["unix_tstamp"] = t.copy()
    if "trhour" not in cols:
        dt = np.asarray(t, np.int64).astype("datetime64[s]")
        days = dt.astype("datetime64[D]")
        secs = (dt - days).astype(np.int64)
        ym = days.astype("datetime64[M]")
        cols["tryear"] = (ym.astype(np.int64) // 12 + 1970).astype(np.int32)
        cols["trmonth"] = (ym.astype(np.int64) % 12 + 1).astype(np.int32)
        cols["trday"] = ((days - ym.astype("datetime64[D]")).astype(np.int64) + 1).astype(np.int32)
        cols["trhour"] = (secs // 3600).astype(np.int32)
        cols["trminute"] = (secs // 60 % 60).astype(np.int32)
        cols["trsec"] = (secs % 60).astype(np.int32)
    out = {}
    for c in schema.FLOW_COLUMNS:
        if c in cols:
            v = cols[c]
        elif c in schema.FLOW_IP_COLUMNS:
            v = np.zeros(n, np.uint32)
        else:
            v = np.zeros(n, np.int64)
        if c in _INT32_COLS:
            v = v.astype(np.int32)
        elif c == "tdur":
            v = v.astype(np.float32)
        out[c] = v
    for c in FLOW_V6_COLUMNS:  # IPv6 endpoints (text), present only when the input had any
        if c in cols:
            out[c] = cols[c]
    return out


def write_flow_csv(path: str, cols: dict, header: bool = True) -> None:
    """ONI flow CSV (inverse of :func:`read_flow_csv`), used by tests and the demo."""
    from .results import ip_str
    n = len(cols["sip"])
    with open(path, "w") as f:
        if header:
            f.write(",".join(c for c, _ in _ONI_FLOW_FIELDS) + "\n")
        for i in range(n):
            row = []
            for c, k in _ONI_FLOW_FIELDS:
                v = cols[c][i]
                if k == TIME:
                    row.append(_dt.datetime.fromtimestamp(int(v), tz=_dt.timezone.utc).strftime("%Y-%m-%d %H:%M:%S"))
                elif k in (IPV4, IPANY):
                    t6 = cols[c + "6"][i] if k == IPANY and (c + "6") in cols else ""
                    row.append(t6 or ip_str(v))
                elif k == F64:
                    row.append(f"{float(v):.3f}")
                else:
                    row.append(str(int(v)))
            f.write(",".join(row) + "\n")


# ------------------------------------------------------------------------------------------------
# Bluecoat proxy logs (C03)
# ------------------------------------------------------------------------------------------------
_BLUECOAT = {  # Bluecoat field name -> (schema column, kind)
    "date": ("p_date", STR), "time": ("p_time", STR), "time-taken": ("duration", I64), "c-ip": ("clientip", IPV4),
    "cs-username": ("username", STR), "cs-auth-group": ("authgroup", STR), "x-exception-id": ("exceptionid", STR),
    "sc-filter-result": ("filterresult", STR), "cs-categories": ("webcat", STR), "cs(referer)": ("referer", STR),
    "sc-status": ("respcode", I64), "s-action": ("action", STR), "cs-method": ("reqmethod", STR),
    "rs(content-type)": ("resconttype", STR), "cs-uri-scheme": ("urischeme", STR), "cs-host": ("host", STR),
    "cs-uri-port": ("uriport", I64), "cs-uri-path": ("uripath", STR), "cs-uri-query": ("uriquery", STR),
    "cs-uri-extension": ("uriextension", STR), "cs(user-agent)": ("useragent", STR), "s-ip": ("serverip", IPV4),
    "sc-bytes": ("scbytes", I64), "cs-bytes": ("csbytes", I64), "x-virus-id": ("virusid", STR),
    "x-bluecoat-application-name": ("bcappname", STR), "x-bluecoat-application-operation": ("bcappoperation", STR),
}


def _gather_strings(buf: np.ndarray, spans: np.ndarray) -> StringColumn:
    b, e = spans[:, 0], spans[:, 1]
    ln = np.maximum(e - b, 0)
    off = np.zeros(len(ln) + 1, np.int64)
    np.cumsum(ln, out=off[1:])
    if off[-1] == 0:
        return StringColumn(off, np.zeros(0, np.uint8))
    idx = np.repeat(b - off[:-1], ln) + np.arange(off[-1])
    return StringColumn(off, buf[idx])


def read_proxy_log(path: str, threads: int = 0) -> dict:
    """Bluecoat access log (``#Fields:`` header defines the order) → proxy-schema columns."""
    from .. import schema
    fields_hdr = None
    with open(path, "rb") as f:
        for raw in f:
            line = raw.decode("utf-8", "replace").strip()
            if line.startswith("#Fields:"):
                fields_hdr = line[len("#Fields:"):].split()
                break
            if line and not line.startswith("#"):
                break
    if fields_hdr is None:
        from ..synth.proxy import PROXY_FIELDS
        fields_hdr = PROXY_FIELDS
    fields = [_BLUECOAT.get(h.lower(), (None, SKIP)) for h in fields_hdr]
    cols, bad = _parse(path, fields, False, sep=" ", threads=threads)
    buf = np.memmap(path, dtype=np.uint8, mode="r") if os.path.getsize(path) else np.zeros(0, np.uint8)
    out = {}
    n = len(next(iter(cols.values()))) if cols else 0
    for c in schema.PROXY_COLUMNS:
        if c in cols:
            v = cols[c]
            out[c] = _gather_strings(np.asarray(buf), v) if v.ndim == 2 else v
        elif c == "fulluri":
            continue
        elif c in ("clientip", "serverip"):
            out[c] = np.zeros(n, np.uint32)
        elif c in ("duration", "respcode", "uriport", "scbytes", "csbytes"):
            out[c] = np.zeros(n, np.int64)
        else:
            out[c] = StringColumn.from_list(["-"] * n)
    for c in ("respcode", "uriport"):
        out[c] = np.asarray(out[c]).astype(np.int32)
    out["fulluri"] = full_uri(out["urischeme"], out["host"], np.asarray(out["uriport"]), out["uripath"],
                              out["uriquery"])
    out["_bad_rows"] = bad
    return out


def _is_dash(c: StringColumn, allow_empty: bool = False) -> np.ndarray:
    ln = np.diff(c.offsets)
    first = np.zeros(len(c), np.uint8)
    nz = ln > 0
    first[nz] = c.chars[c.offsets[:-1][nz]]
    m = (ln == 1) & (first == ord("-"))
    return m | (ln == 0) if allow_empty else m


def full_uri(scheme: StringColumn, host: StringColumn, port: np.ndarray, path: StringColumn,
             query: StringColumn) -> StringColumn:
    """``scheme://host[:port]path[query]`` per row (port omitted for 0/80/443, '-' fields
    dropped), vectorised (StringColumn.join_rows) -- no per-row Python at 1e8 rows."""
    port = np.asarray(port).astype(np.int64)
    up, inv = np.unique(port, return_inverse=True)
    pstr = StringColumn.from_list([f":{p}" for p in up.tolist()]).take(inv)
    return StringColumn.join_rows([(scheme, None), (b"://", None), (host, None),
                                   (pstr, ~np.isin(port, (0, 80, 443))), (path, ~_is_dash(path)),
                                   (query, ~_is_dash(query, allow_empty=True))])


_MONTHS = np.frombuffer(b"JanFebMarAprMayJunJulAugSepOctNovDec", np.uint8).reshape(12, 3)
_DIGITS2 = np.frombuffer("".join(f"{i:02d}" for i in range(100)).encode(), np.uint8).reshape(100, 2)


def frame_times(ts_ns: np.ndarray) -> StringColumn:
    """tshark ``frame.time`` text ("%b %d, %Y %H:%M:%S.%f UTC", fixed 32 bytes) of nanosecond
    timestamps, vectorised (numpy datetime64 fields + digit arithmetic)."""
    ts_ns = np.asarray(ts_ns, np.int64)
    n = ts_ns.size
    us = ts_ns // 1000
    dt = us.astype("datetime64[us]")
    day = dt.astype("datetime64[D]")
    ym = dt.astype("datetime64[M]")
    year = ym.astype(np.int64) // 12 + 1970
    month = ym.astype(np.int64) % 12
    mday = (day - ym.astype("datetime64[D]")).astype(np.int64) + 1
    sod = us - day.astype("datetime64[us]").astype(np.int64)
    hh, mm, ss, frac = sod // 3_600_000_000, sod // 60_000_000 % 60, sod // 1_000_000 % 60, sod % 1_000_000
    out = np.empty((n, 32), np.uint8)

    def put(col, v, w):  # w-digit zero-padded decimal (w even) via a two-digit table
        for k in range(0, w, 2):
            out[:, col + w - 2 - k:col + w - k] = _DIGITS2[(v // 10 ** k) % 100]

    out[:, 0:3] = _MONTHS[month]
    out[:, 3] = 32
    put(4, mday, 2)
    out[:, 6], out[:, 7] = 44, 32
    put(8, year, 4)
    out[:, 12] = 32
    put(13, hh, 2)
    out[:, 15] = 58
    put(16, mm, 2)
    out[:, 18] = 58
    put(19, ss, 2)
    out[:, 21] = 46
    put(22, frac, 6)
    out[:, 28:32] = np.frombuffer(b" UTC", np.uint8)
    return StringColumn.from_fixed(out)


class FrameTimeColumn(StringColumn):
    """``frame_time`` of a decoded pcap, formatted lazily: the ML path never reads the text (it
    uses ``unix_tstamp``), so only the rows that are rendered (the top-N results) or stored are
    ever formatted (:func:`frame_times`). Behaves as a StringColumn everywhere else."""

    def __init__(self, ts_ns: np.ndarray):  # noqa: super().__init__ deliberately not called
        self.ts_ns = np.asarray(ts_ns, np.int64)
        self._mat = None

    def _m(self) -> StringColumn:
        if self._mat is None:
            self._mat = frame_times(self.ts_ns)
        return self._mat

    offsets = property(lambda self: self._m().offsets)
    chars = property(lambda self: self._m().chars)

    def __len__(self) -> int:
        return int(self.ts_ns.size)

    def take(self, idx) -> StringColumn:
        return frame_times(self.ts_ns[np.asarray(idx, dtype=np.int64)])

    def slice(self, lo: int, hi: int) -> "FrameTimeColumn":
        return FrameTimeColumn(self.ts_ns[lo:hi])


# ------------------------------------------------------------------------------------------------
# pcap DNS
# ------------------------------------------------------------------------------------------------
def read_pcap_dns(path: str, threads: int = 0) -> dict:
    L = native.lib()
    h = L.oni_pcap_dns_open(path.encode(), threads)
    try:
        rows, nb, ab, pk = (C.c_int64() for _ in range(4))
        rc = L.oni_pcap_dns_sizes(h, C.byref(rows), C.byref(nb), C.byref(ab), C.byref(pk))
        if rc != 0:
            raise OSError(f"cannot decode {path}")
        n = rows.value
        ts = np.empty(n, np.int64)
        flen = np.empty(n, np.int32)
        src = np.empty(n, np.uint32)
        dst = np.empty(n, np.uint32)
        qt = np.empty(n, np.int32)
        qc = np.empty(n, np.int32)
        rc_ = np.empty(n, np.int32)
        noff = np.empty(n + 1, np.int64)
        names = np.empty(max(nb.value, 1), np.uint8)
        aoff = np.empty(n + 1, np.int64)
        aa = np.empty(max(ab.value, 1), np.uint8)
        L.oni_pcap_dns_fetch(h, *(x.ctypes.data for x in (ts, flen, src, dst, qt, qc, rc_, noff, names, aoff, aa)))
        st = np.zeros(2, np.int64)
        L.oni_pcap_dns_stats(h, st.ctypes.data)
    finally:
        L.oni_pcap_dns_free(h)
    unix = ts // 1_000_000_000
    return {
        "frame_time": FrameTimeColumn(ts),
        "unix_tstamp": unix,
        "frame_len": flen,
        "ip_src": src,
        "ip_dst": dst,
        "dns_qry_name": StringColumn(noff, names[: nb.value]),
        "dns_qry_type": qt,
        "dns_qry_class": qc,
        "dns_qry_rcode": rc_,
        "dns_a": StringColumn(aoff, aa[: ab.value]),
        "_packets": pk.value,
        "_tcp_partial": int(st[0]),       # DNS-over-TCP messages split across segments (skipped)
        "_frag_incomplete": int(st[1]),   # IPv4 datagrams with missing fragments (skipped)
    }


def write_pcap_dns(path: str, ts_ns, ip_server, ip_client, names: StringColumn, qtype, rcode, n_answers=None,
                   answer_ip=None, pad_to: int = 0) -> int:
    n = len(names)
    arrs = [np.ascontiguousarray(a, dt) for a, dt in ((ts_ns, np.int64), (ip_server, np.uint32),
                                                       (ip_client, np.uint32), (names.offsets, np.int64),
                                                       (names.chars, np.uint8), (qtype, np.int32),
                                                       (rcode, np.int32))]
    na = np.ascontiguousarray(n_answers if n_answers is not None else np.zeros(n), np.int32)
    ai = np.ascontiguousarray(answer_ip if answer_ip is not None else np.zeros(n), np.uint32)
    r = native.lib().oni_pcap_dns_write(path.encode(), n, *(a.ctypes.data for a in arrs), na.ctypes.data,
                                        ai.ctypes.data, pad_to)
    if r != n:
        raise OSError(f"pcap write failed: {path}")
    return r
