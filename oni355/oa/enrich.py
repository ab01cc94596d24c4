"""Operational-analytics enrichment (oni-oa flow_oa.py / dns_oa.py / proxy_oa.py; SURVEY.md
§2.2 C27-C31, [U-M]): turn an ML results CSV into the analyst's ``<source>_scores.csv`` with
geo-location, network context, reputation and IANA code names, ``sev = 0`` (unscored).

* Geo (C28): IP-range table CSV ``start_ip,end_ip,location`` (integers or dotted), vectorised
  ``searchsorted`` on the range starts.
* Network context (C29): CSV ``cidr_or_range,name`` → internal flag + name.
* Reputation (C30): pluggable services (:mod:`oni355.oa.reputation`).
* IANA (C31): DNS qtype/qclass/rcode and HTTP status names (:mod:`oni355.oa.iana`).
"""
from __future__ import annotations

import csv
import ipaddress
import os

import numpy as np

from .. import schema
from ..io import results as rio
from . import iana
from .reputation import ReputationService


def _ip_int(s: str) -> int:
    s = s.strip()
    if s.isdigit():
        return int(s)
    try:
        return int(ipaddress.IPv4Address(s))
    except ValueError:
        return 0


class RangeTable:
    """Sorted, non-overlapping [start, end] → label table (geo / network context)."""

    def __init__(self, starts, ends, labels):
        o = np.argsort(np.asarray(starts, np.int64), kind="stable")
        self.starts = np.asarray(starts, np.int64)[o]
        self.ends = np.asarray(ends, np.int64)[o]
        self.labels = [labels[i] for i in o]

    @classmethod
    def from_csv(cls, path: str) -> "RangeTable":
        starts, ends, labels = [], [], []
        with open(path, newline="") as f:
            for row in csv.reader(f):
                if not row or row[0].startswith("#"):
                    continue
                if "/" in row[0]:
                    net = ipaddress.IPv4Network(row[0].strip(), strict=False)
                    starts.append(int(net.network_address))
                    ends.append(int(net.broadcast_address))
                    labels.append(row[1].strip() if len(row) > 1 else "")
                else:
                    if len(row) < 2 or not row[0].strip()[0].isdigit():
                        continue
                    starts.append(_ip_int(row[0]))
                    ends.append(_ip_int(row[1]))
                    labels.append(",".join(x.strip() for x in row[2:]) if len(row) > 2 else "")
        return cls(starts, ends, labels)

    def lookup(self, ips) -> list[str]:
        ips = np.asarray(ips, np.int64)
        if self.starts.size == 0:
            return [""] * ips.size
        i = np.searchsorted(self.starts, ips, side="right") - 1
        ok = (i >= 0) & (ips <= self.ends[np.clip(i, 0, None)])
        return [self.labels[j] if k else "" for j, k in zip(i.tolist(), ok.tolist())]


DEFAULT_INTERNAL = [("10.0.0.0/8", "internal"), ("172.16.0.0/12", "internal"), ("192.168.0.0/16", "internal")]


def default_context() -> RangeTable:
    s, e, lab = [], [], []
    for cidr, name in DEFAULT_INTERNAL:
        n = ipaddress.IPv4Network(cidr)
        s.append(int(n.network_address))
        e.append(int(n.broadcast_address))
        lab.append(name)
    return RangeTable(s, e, lab)


def enrich(source: str, results_csv: str, out_csv: str, limit: int | None = None, geo: RangeTable | None = None,
           context: RangeTable | None = None, reputation: list[ReputationService] | None = None) -> int:
    """Results CSV → scores CSV (the OA start step). Returns rows written."""
    header, rows = rio.read_csv(results_csv)
    if limit:
        rows = rows[:limit]
    ix = {h: i for i, h in enumerate(header)}
    ctx = context or default_context()
    rep = reputation or []
    out = []
    if source == "flow":
        sips = [_ip_int(r[ix["sip"]]) for r in rows]
        dips = [_ip_int(r[ix["dip"]]) for r in rows]
        sgeo = geo.lookup(sips) if geo else [""] * len(rows)
        dgeo = geo.lookup(dips) if geo else [""] * len(rows)
        sctx, dctx = ctx.lookup(sips), ctx.lookup(dips)
        srep = _rep(rep, [r[ix["sip"]] for r in rows])
        drep = _rep(rep, [r[ix["dip"]] for r in rows])
        for i, r in enumerate(rows):
            out.append(["0", r[ix["treceived"]], r[ix["sip"]], r[ix["dip"]], r[ix["sport"]], r[ix["dport"]],
                        r[ix["proto"]], r[ix["ipkt"]], r[ix["ibyt"]], sgeo[i], dgeo[i], sctx[i], dctx[i], srep[i],
                        drep[i]])
    elif source == "dns":
        from ..ref.strings_spec import entropy, split_domain
        ips = [_ip_int(r[ix["ip_dst"]]) for r in rows]
        nctx = ctx.lookup(ips)
        qrep = _rep(rep, [r[ix["dns_qry_name"]] for r in rows])
        for i, r in enumerate(rows):
            name = r[ix["dns_qry_name"]].encode()
            reg, b, per = split_domain(name)
            sub = name[: reg - 1] if reg > 0 else b""
            qt, qc, rc = (int(float(r[ix[c]] or 0)) for c in ("dns_qry_type", "dns_qry_class", "dns_qry_rcode"))
            out.append(["0", r[ix["frame_time"]], r[ix["frame_len"]], r[ix["ip_dst"]], r[ix["dns_qry_name"]],
                        str(qc), str(qt), str(rc), name[reg:b].decode(), sub.decode(), str(len(sub)), str(per),
                        f"{float(entropy(sub)):.6f}", r[ix["word"]].split("_")[0], r[ix["word"]], r[ix["score"]],
                        qrep[i], "", "0", "0", iana.dns_class(qc), iana.dns_type(qt), iana.dns_rcode(rc), nctx[i],
                        r[ix["unix_tstamp"]]])
    else:
        ips = [_ip_int(r[ix["clientip"]]) for r in rows]
        nctx = ctx.lookup(ips)
        urep = _rep(rep, [r[ix["fulluri"]] for r in rows])
        keep = [c for c in schema.PROXY_SCORE_COLUMNS[1:] if c in ix]
        for i, r in enumerate(rows):
            rec = {c: r[ix[c]] for c in keep}
            rec.update({"uri_rep": urep[i], "respcode_name": iana.http_status(int(float(r[ix["respcode"]] or 0))),
                        "network_context": nctx[i]})
            out.append(["0"] + [rec.get(c, "") for c in schema.PROXY_SCORE_COLUMNS[1:]])
    rio.write_csv(out_csv, schema.score_columns(source), out)
    return len(out)


def _rep(services: list[ReputationService], keys: list[str]) -> list[str]:
    if not services:
        return [""] * len(keys)
    uniq = sorted(set(keys))
    res = {k: [] for k in uniq}
    for s in services:
        for k, v in s.check(uniq).items():
            if v:
                res[k].append(f"{s.name}:{v}")
    return ["::".join(res[k]) for k in keys]


def default_paths(lpath: str, source: str, date: str) -> tuple[str, str]:
    return rio.results_path(lpath, source, date), os.path.join(lpath, source, date, f"{source}_scores.csv")
