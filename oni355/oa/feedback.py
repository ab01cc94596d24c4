"""Analyst feedback ("noise filter").

The OA side writes ``<source>_scores.csv`` (first column ``sev``: 0 unscored, 1 high, 2 medium,
3 low/benign). The next ``oni-ml`` run reads rows with ``sev == 3``, re-words them with the new
day's cuts and adds each word DUPFACTOR times to its IP document, so the pattern becomes normal.

* :func:`load_feedback` -- scores CSV → feedback columns for the ML pipelines
* :func:`set_severity`  -- analyst action: mark rows (by IP / word / row index) with a severity
"""
from __future__ import annotations

import csv
import datetime as _dt
import os

import numpy as np

from .. import schema
from ..store.columnar import StringColumn


def _ip(s: str) -> int:
    try:
        a, b, c, d = (int(x) for x in s.strip().split("."))
        return (a << 24) | (b << 16) | (c << 8) | d
    except ValueError:
        return 0


def _read(path: str) -> tuple[list[str], list[list[str]]]:
    with open(path, newline="") as f:
        r = csv.reader(f)
        header = next(r, [])
        return header, [row for row in r if row]


def load_feedback(path: str, source: str, sev: int = schema.SEV_LOW) -> dict | None:
    header, rows = _read(path)
    if not header or "sev" not in header:
        return None
    ix = {h: i for i, h in enumerate(header)}
    sel = [r for r in rows if r[ix["sev"]].strip() and int(float(r[ix["sev"]])) == sev]
    if not sel:
        return None

    def col(name, default=""):
        return [r[ix[name]] if name in ix and ix[name] < len(r) else default for r in sel]

    if source == "flow":
        ts = [_dt.datetime.strptime(t.strip()[:19], "%Y-%m-%d %H:%M:%S") for t in col("tstart", "1970-01-01 00:00:00")]
        v6 = {}
        for c, name in (("srcIP", "sip6"), ("dstIP", "dip6")):
            txt = [x.strip() if ":" in x else "" for x in col(c)]
            if any(txt):  # IPv6 endpoints: keyed by the pipeline's day dictionary (flow.with_ipv6_keys)
                v6[name] = StringColumn.from_list(txt)
        return {**v6,
            "trhour": np.array([t.hour for t in ts], np.int32), "trminute": np.array([t.minute for t in ts], np.int32),
            "trsec": np.array([t.second for t in ts], np.int32),
            "sip": np.array([_ip(x) for x in col("srcIP")], np.uint32),
            "dip": np.array([_ip(x) for x in col("dstIP")], np.uint32),
            "sport": np.array([int(float(x or 0)) for x in col("sport")], np.int32),
            "dport": np.array([int(float(x or 0)) for x in col("dport")], np.int32),
            "ipkt": np.array([int(float(x or 0)) for x in col("ipkt")], np.int64),
            "ibyt": np.array([int(float(x or 0)) for x in col("ibyt")], np.int64),
        }
    if source == "dns":
        return {
            "unix_tstamp": np.array([int(float(x or 0)) for x in col("unix_tstamp")], np.int64),
            "frame_len": np.array([int(float(x or 0)) for x in col("frame_len")], np.int32),
            "ip_dst": np.array([_ip(x) for x in col("ip_dst")], np.uint32),
            "dns_qry_name": StringColumn.from_list(col("dns_qry_name")),
            "dns_qry_type": np.array([int(float(x or 0)) for x in col("dns_qry_type")], np.int32),
            "dns_qry_rcode": np.array([int(float(x or 0)) for x in col("dns_qry_rcode")], np.int32),
        }
    return {
        "clientip": np.array([_ip(x) for x in col("clientip")], np.uint32),
        "host": StringColumn.from_list(col("host")), "p_time": StringColumn.from_list(col("p_time", "00:00:00")),
        "useragent": StringColumn.from_list(col("useragent")), "fulluri": StringColumn.from_list(col("fulluri")),
        "reqmethod": StringColumn.from_list(col("reqmethod")),
        "resconttype": StringColumn.from_list(col("resconttype")),
        "respcode": np.array([int(float(x or 0)) for x in col("respcode")], np.int32),
    }


def set_severity(path: str, sev: int, ip: str | None = None, word: str | None = None, rows=None) -> int:
    """Mark matching rows of a scores file with ``sev``; returns how many rows changed."""
    header, data = _read(path)
    ix = {h: i for i, h in enumerate(header)}
    ip_cols = [c for c in ("srcIP", "dstIP", "ip_dst", "clientip") if c in ix]
    changed = 0
    rowset = set(rows) if rows is not None else None
    for i, r in enumerate(data):
        hit = rowset is not None and i in rowset
        if ip is not None and any(r[ix[c]] == ip for c in ip_cols):
            hit = True
        if word is not None and "word" in ix and r[ix["word"]] == word:
            hit = True
        if hit and r[ix["sev"]] != str(sev):
            r[ix["sev"]] = str(sev)
            changed += 1
    tmp = path + ".tmp"
    with open(tmp, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(data)
    os.replace(tmp, path)
    return changed
