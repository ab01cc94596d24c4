"""OA detail queries (oni-oa components/data impala/hive queries; SURVEY.md §2.2 C32, [U-M]).

The reference issued Impala queries per analyst click (edge details, chord diagrams, time series,
ingest summary) and wrote ``edge-*.tsv`` / ``chord-*.tsv``. Here the same questions are column
filters over the day's columnar store (or any loaded column dict).
"""
from __future__ import annotations

import csv
import glob
import os

import numpy as np

from ..io.results import ip_str
from ..store import columnar


def _ip(s) -> int:
    if isinstance(s, (int, np.integer)):
        return int(s)
    a, b, c, d = (int(x) for x in str(s).split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def _is_v6(ip) -> bool:
    return isinstance(ip, str) and ":" in ip


def ip_mask(cols: dict, col: str, ip) -> np.ndarray:
    """Rows whose ``col`` endpoint is ``ip`` (IPv6 text matches the ``<col>6`` text column)."""
    if _is_v6(ip):
        c6 = cols.get(col + "6")
        return str_eq_mask(c6, ip) if c6 is not None else np.zeros(len(cols[col]), bool)
    m = np.asarray(cols[col], np.uint32) == _ip(ip)
    if col + "6" in cols:
        m &= np.diff(cols[col + "6"].offsets) == 0  # an IPv6 row's u32 column is 0, not an address
    return m


def _ip_texts(cols: dict, col: str, idx: np.ndarray) -> list[str]:
    v4 = [ip_str(x) for x in np.asarray(cols[col])[idx]]
    if col + "6" not in cols:
        return v4
    return [t or a for t, a in zip(cols[col + "6"].take(idx).to_list(), v4)]


def edge_details(cols: dict, src_ip, dst_ip, hour: int | None = None, limit: int = 1000) -> list[dict]:
    """All flows between two hosts (either direction, IPv4 or IPv6), optionally within one hour."""
    m = ((ip_mask(cols, "sip", src_ip) & ip_mask(cols, "dip", dst_ip))
         | (ip_mask(cols, "sip", dst_ip) & ip_mask(cols, "dip", src_ip)))
    if hour is not None:
        m &= np.asarray(cols["trhour"]) == hour
    idx = np.nonzero(m)[0][:limit]
    keys = ["unix_tstamp", "sip", "dip", "sport", "dport", "proto", "ipkt", "ibyt", "opkt", "obyt", "tdur"]
    txt = {c: _ip_texts(cols, c, idx) for c in ("sip", "dip")}
    out = []
    for j, i in enumerate(idx):
        rec = {k: (txt[k][j] if k in ("sip", "dip") else cols[k][i].item()) for k in keys if k in cols}
        out.append(rec)
    return out


def chord(cols: dict, ip, top: int = 50) -> list[tuple[str, str, int, int]]:
    """Bytes/packets exchanged between ``ip`` and each peer (the chord-diagram query)."""
    ms, md = ip_mask(cols, "sip", ip), ip_mask(cols, "dip", ip)
    m = ms | md
    idx = np.nonzero(m)[0]
    if idx.size == 0:
        return []
    s_txt, d_txt = _ip_texts(cols, "sip", idx), _ip_texts(cols, "dip", idx)
    peer = np.array([d if a else s for a, s, d in zip(ms[idx], s_txt, d_txt)], dtype=object)
    byt = np.asarray(cols["ibyt"], np.int64)[idx]
    pkt = np.asarray(cols["ipkt"], np.int64)[idx]
    up, inv = np.unique(peer.astype(str), return_inverse=True)
    b = np.bincount(inv, weights=byt).astype(np.int64)
    p = np.bincount(inv, weights=pkt).astype(np.int64)
    order = np.argsort(-b, kind="stable")[:top]
    me = ip if _is_v6(ip) else ip_str(_ip(ip))
    return [(me, str(up[i]), int(b[i]), int(p[i])) for i in order]


def timeline(cols: dict, ip, bucket_s: int = 3600) -> list[tuple[int, int]]:
    """Events per time bucket for one IP (flow: either endpoint; dns: client; proxy: client)."""
    if "sip" in cols:
        m = ip_mask(cols, "sip", ip) | ip_mask(cols, "dip", ip)
    elif "ip_dst" in cols:
        x = _ip(ip)
        m = np.asarray(cols["ip_dst"], np.uint32) == x
    else:
        m = np.asarray(cols["clientip"], np.uint32) == _ip(ip)
    if "unix_tstamp" in cols:
        t = np.asarray(cols["unix_tstamp"], np.int64)[m] // bucket_s * bucket_s
    else:  # proxy logs carry p_date/p_time only: hour-of-day buckets (seconds into the day)
        t = event_hours(cols, "proxy")[m] * 3600 // bucket_s * bucket_s
    u, c = np.unique(t, return_counts=True)
    return list(zip(u.tolist(), c.tolist()))


def ingest_summary(root: str, source: str, date: str) -> list[tuple[int, int]]:
    """Events per hour of a stored day (the OA ingest-summary page); hour partitions are counted
    from their metadata without reading any column."""
    hs = columnar.hours(root, source, date)
    if hs and not os.path.exists(os.path.join(columnar.day_dir(root, source, date), "_schema.json")) and \
            not glob.glob(os.path.join(columnar.day_dir(root, source, date), "part-*")):
        c = {h: columnar.rows(root, source, date, hours=[h]) for h in hs}
        return [(i, int(c.get(i, 0))) for i in range(24)]
    cols = columnar.read_day(root, source, date, columns=["unix_tstamp"] if source != "proxy" else ["p_time"])
    return ingest_summary_cols(cols, source)


def write_tsv(path: str, header: list[str], rows) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f, delimiter="\t")
        w.writerow(header)
        for r in rows:
            w.writerow(list(r.values()) if isinstance(r, dict) else list(r))
    return path


# ------------------------------------------------------------------------------------------------
# per-suspicious-row detail files (oni-oa "details": edge / chord / dendrogram / timeline TSVs)
# ------------------------------------------------------------------------------------------------
def str_eq_mask(col, s: str) -> np.ndarray:
    """Rows of a StringColumn equal to ``s`` (case-insensitive), vectorised: length filter, then
    one [candidates × len] byte comparison."""
    b = np.frombuffer(s.lower().encode(), np.uint8)
    ln = np.diff(col.offsets)
    cand = np.nonzero(ln == b.size)[0]
    m = np.zeros(len(col), bool)
    if cand.size == 0:
        return m
    if b.size == 0:
        m[cand] = True
        return m
    g = col.chars[col.offsets[cand][:, None] + np.arange(b.size)[None, :]]
    g = np.where((g >= 65) & (g <= 90), g + 32, g)
    m[cand[(g == b[None, :]).all(1)]] = True
    return m


def event_hours(cols: dict, source: str) -> np.ndarray:
    if source == "flow" and "trhour" in cols:
        return np.asarray(cols["trhour"], np.int64)
    if source == "proxy":
        from ..ingest.watch import _fixed_digits
        return _fixed_digits(cols["p_time"], [0, 1])
    return (np.asarray(cols["unix_tstamp"], np.int64) % 86400) // 3600


def ingest_summary_cols(cols: dict, source: str) -> list[tuple[int, int]]:
    c = np.bincount(np.clip(event_hours(cols, source), 0, 23), minlength=24)
    return [(i, int(c[i])) for i in range(24)]


def dns_edge(cols: dict, qname: str, hour: int | None = None, limit: int = 1000) -> list[tuple]:
    """Every query for one name (optionally within one hour) -- the DNS edge view."""
    m = str_eq_mask(cols["dns_qry_name"], qname)
    if hour is not None:
        m &= event_hours(cols, "dns") == hour
    idx = np.nonzero(m)[0][:limit]
    names, ans = cols["dns_qry_name"].take(idx).to_list(), cols["dns_a"].take(idx).to_list() if "dns_a" in cols else \
        [""] * idx.size
    t = np.asarray(cols["unix_tstamp"], np.int64)
    return [(int(t[i]), ip_str(cols["ip_src"][i]), ip_str(cols["ip_dst"][i]), names[j],
             int(cols["dns_qry_type"][i]), int(cols["dns_qry_rcode"][i]), ans[j]) for j, i in enumerate(idx)]


def dns_dendro(cols: dict, ip, top: int = 200) -> list[tuple[str, str, int]]:
    """(registered domain, subdomain, queries) for one client IP -- the DNS dendrogram query."""
    from ..ref.strings_spec import split_domain
    x = _ip(ip)
    idx = np.nonzero(np.asarray(cols["ip_dst"], np.uint32) == x)[0]
    cnt: dict = {}
    for name in cols["dns_qry_name"].take(idx).to_list():
        b = name.encode()
        r, e, _ = split_domain(b)
        key = (b[r:e].decode(), b[: r - 1].decode() if r > 0 else "")
        cnt[key] = cnt.get(key, 0) + 1
    return sorted(((d, s, c) for (d, s), c in cnt.items()), key=lambda t: (-t[2], t[0], t[1]))[:top]


def proxy_edge(cols: dict, clientip, host: str, hour: int | None = None, limit: int = 1000) -> list[tuple]:
    """Requests of one client to one host (optionally within one hour) -- the proxy edge view."""
    x = _ip(clientip)
    m = (np.asarray(cols["clientip"], np.uint32) == x) & str_eq_mask(cols["host"], host)
    if hour is not None:
        m &= event_hours(cols, "proxy") == hour
    idx = np.nonzero(m)[0][:limit]
    get = {c: cols[c].take(idx).to_list() for c in ("p_date", "p_time", "reqmethod", "useragent", "fulluri")
           if c in cols}
    out = []
    for j, i in enumerate(idx):
        out.append((get["p_date"][j], get["p_time"][j], ip_str(cols["clientip"][i]), host, get["reqmethod"][j],
                    get["useragent"][j], int(cols["respcode"][i]), get["fulluri"][j], int(cols["scbytes"][i]),
                    int(cols["csbytes"][i])))
    return out


EDGE_HEADERS = {
    "flow": ["unix_tstamp", "sip", "dip", "sport", "dport", "proto", "ipkt", "ibyt", "opkt", "obyt", "tdur"],
    "dns": ["unix_tstamp", "ip_src", "ip_dst", "dns_qry_name", "dns_qry_type", "dns_qry_rcode", "dns_a"],
    "proxy": ["p_date", "p_time", "clientip", "host", "reqmethod", "useragent", "respcode", "fulluri", "scbytes",
              "csbytes"],
}


def _safe(s: str) -> str:
    """File-name form of an IP / name (IPv6 ':' would read as a URL scheme in the pages' links)."""
    return "".join(c if c.isalnum() or c in ".-_" else "_" for c in s)[:120]


def write_details(source: str, results_csv: str, cols: dict, out_dir: str, limit: int = 10) -> dict:
    """Detail TSVs for the ``limit`` most suspicious result rows (the reference's per-row
    ``edge-*.tsv`` / ``chord-*.tsv`` / dendrogram / timeline files + the ingest summary); returns
    the index that the static pages (oni355.oa.pages) read, also written as ``index.json``."""
    import json
    from ..io import results as rio
    header, rows = rio.read_csv(results_csv)
    ix = {h: i for i, h in enumerate(header)}
    os.makedirs(out_dir, exist_ok=True)
    index = {"source": source, "rows": [], "ips": {}}
    index["ingest_summary"] = os.path.basename(write_tsv(os.path.join(out_dir, "ingest_summary.tsv"),
                                                         ["hour", "events"], ingest_summary_cols(cols, source)))

    def per_ip(ip: str) -> None:
        if ip in index["ips"]:
            return
        ent = {"page": f"threat-{_safe(ip)}.html", "timeline": os.path.basename(write_tsv(os.path.join(out_dir, f"timeline-{_safe(ip)}.tsv"),
                                                      ["bucket_start", "events"], timeline(cols, ip)))}
        if source == "flow":
            ent["chord"] = os.path.basename(write_tsv(os.path.join(out_dir, f"chord-{_safe(ip)}.tsv"),
                                                      ["ip", "peer", "bytes", "packets"], chord(cols, ip)))
        elif source == "dns":
            ent["dendro"] = os.path.basename(write_tsv(os.path.join(out_dir, f"dendro-{_safe(ip)}.tsv"),
                                                       ["domain", "subdomain", "queries"], dns_dendro(cols, ip)))
        index["ips"][ip] = ent

    for rank, r in enumerate(rows[:limit]):
        if source == "flow":
            sip, dip, hh = r[ix["sip"]], r[ix["dip"]], int(r[ix["trhour"]])
            e = edge_details(cols, sip, dip, hour=hh)
            f = write_tsv(os.path.join(out_dir, f"edge-{_safe(sip)}-{_safe(dip)}-{hh:02d}.tsv"), EDGE_HEADERS["flow"], e)
            ip, peer = sip, dip
            per_ip(sip)
            per_ip(dip)
        elif source == "dns":
            ip, peer = r[ix["ip_dst"]], r[ix["dns_qry_name"]]
            hh = int(int(float(r[ix["unix_tstamp"]])) % 86400 // 3600)
            e = dns_edge(cols, peer, hour=hh)
            f = write_tsv(os.path.join(out_dir, f"edge-{_safe(peer)}-{hh:02d}.tsv"), EDGE_HEADERS["dns"], e)
            per_ip(ip)
        else:
            ip, peer = r[ix["clientip"]], r[ix["host"]]
            hh = int(r[ix["p_time"]][:2] or 0)
            e = proxy_edge(cols, ip, peer, hour=hh)
            f = write_tsv(os.path.join(out_dir, f"edge-{ip}-{_safe(peer)}-{hh:02d}.tsv"), EDGE_HEADERS["proxy"], e)
            per_ip(ip)
        index["rows"].append({"rank": rank, "ip": ip, "peer": peer, "hour": hh, "edge": os.path.basename(f),
                              "edge_rows": len(e), "score": r[ix["score"]]})
    with open(os.path.join(out_dir, "index.json"), "w") as fh:
        json.dump(index, fh, indent=1)
    return index
