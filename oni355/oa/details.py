"""OA detail queries (oni-oa components/data impala/hive queries; SURVEY.md §2.2 C32, [U-M]).

The reference issued Impala queries per analyst click (edge details, chord diagrams, time series,
ingest summary) and wrote ``edge-*.tsv`` / ``chord-*.tsv``. Here the same questions are column
filters over the day's columnar store (or any loaded column dict).
"""
from __future__ import annotations

import csv
import os

import numpy as np

from ..io.results import ip_str
from ..store import columnar


def _ip(s) -> int:
    if isinstance(s, (int, np.integer)):
        return int(s)
    a, b, c, d = (int(x) for x in str(s).split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def edge_details(cols: dict, src_ip, dst_ip, hour: int | None = None, limit: int = 1000) -> list[dict]:
    """All flows between two hosts (either direction), optionally within one hour."""
    s, d = _ip(src_ip), _ip(dst_ip)
    sip, dip = np.asarray(cols["sip"], np.uint32), np.asarray(cols["dip"], np.uint32)
    m = ((sip == s) & (dip == d)) | ((sip == d) & (dip == s))
    if hour is not None:
        m &= np.asarray(cols["trhour"]) == hour
    idx = np.nonzero(m)[0][:limit]
    keys = ["unix_tstamp", "sip", "dip", "sport", "dport", "proto", "ipkt", "ibyt", "opkt", "obyt", "tdur"]
    out = []
    for i in idx:
        rec = {k: (ip_str(cols[k][i]) if k in ("sip", "dip") else cols[k][i].item()) for k in keys if k in cols}
        out.append(rec)
    return out


def chord(cols: dict, ip, top: int = 50) -> list[tuple[str, str, int, int]]:
    """Bytes/packets exchanged between ``ip`` and each peer (the chord-diagram query)."""
    x = _ip(ip)
    sip, dip = np.asarray(cols["sip"], np.uint32), np.asarray(cols["dip"], np.uint32)
    m = (sip == x) | (dip == x)
    peer = np.where(sip[m] == x, dip[m], sip[m])
    byt = np.asarray(cols["ibyt"], np.int64)[m]
    pkt = np.asarray(cols["ipkt"], np.int64)[m]
    if peer.size == 0:
        return []
    up, inv = np.unique(peer, return_inverse=True)
    b = np.bincount(inv, weights=byt).astype(np.int64)
    p = np.bincount(inv, weights=pkt).astype(np.int64)
    order = np.argsort(-b, kind="stable")[:top]
    return [(ip_str(x), ip_str(up[i]), int(b[i]), int(p[i])) for i in order]


def timeline(cols: dict, ip, bucket_s: int = 3600) -> list[tuple[int, int]]:
    """Events per time bucket for one IP (flow: either endpoint; dns: client; proxy: client)."""
    x = _ip(ip)
    if "sip" in cols:
        m = (np.asarray(cols["sip"], np.uint32) == x) | (np.asarray(cols["dip"], np.uint32) == x)
    elif "ip_dst" in cols:
        m = np.asarray(cols["ip_dst"], np.uint32) == x
    else:
        m = np.asarray(cols["clientip"], np.uint32) == x
    t = np.asarray(cols["unix_tstamp"], np.int64)[m] // bucket_s * bucket_s
    u, c = np.unique(t, return_counts=True)
    return list(zip(u.tolist(), c.tolist()))


def ingest_summary(root: str, source: str, date: str) -> list[tuple[int, int]]:
    """Events per hour of a stored day (the OA ingest-summary page)."""
    cols = columnar.read_day(root, source, date, columns=["unix_tstamp"] if source != "proxy" else ["p_time"])
    if source == "proxy":
        h = np.array([int(s[:2]) if s else 0 for s in cols["p_time"].to_list()], np.int64)
    else:
        h = (np.asarray(cols["unix_tstamp"], np.int64) % 86400) // 3600
    c = np.bincount(h, minlength=24)
    return [(i, int(c[i])) for i in range(24)]


def write_tsv(path: str, header: list[str], rows) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f, delimiter="\t")
        w.writerow(header)
        for r in rows:
            w.writerow(list(r.values()) if isinstance(r, dict) else list(r))
    return path
