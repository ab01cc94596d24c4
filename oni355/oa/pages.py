"""Static analyst pages (the oni-oa web UI's views; reference README
"Visualization" / "Attack heuristics"): suspicious connects, threat investigation, storyboard and
ingest summary, rendered as self-contained HTML with inline SVG (no server, no JS libraries, no
network). Input: the day's ``<source>_scores.csv`` (oni-oa enrich), the ``details/`` TSVs +
``index.json`` (oni-oa details) and ``threats.json`` (oni-oa threat).
"""
from __future__ import annotations

import csv
import html
import json
import math
import os

SEV_COLORS = {"0": "#ffffff", "1": "#f8d0d0", "2": "#fbe8c0", "3": "#d8f0d8"}
_CSS = ("body{font-family:sans-serif;margin:1.5em}table{border-collapse:collapse;font-size:12px}"
        "td,th{border:1px solid #bbb;padding:2px 6px}th{background:#eee}h1{font-size:20px}h2{font-size:16px}"
        "nav a{margin-right:1em}.bar{fill:#4a78b0}.axis{font-size:10px}")


def _read_tsv(path: str) -> tuple[list[str], list[list[str]]]:
    if not os.path.exists(path):
        return [], []
    with open(path, newline="") as f:
        r = list(csv.reader(f, delimiter="\t"))
    return (r[0], r[1:]) if r else ([], [])


def _page(title: str, body: str, source: str, date: str) -> str:
    nav = "".join(f'<a href="{p}.html">{t}</a>' for p, t in (("suspicious", "Suspicious"), ("storyboard", "Storyboard"),
                                                             ("ingest_summary", "Ingest summary")))
    return (f"<!doctype html><html><head><meta charset='utf-8'><title>{html.escape(title)}</title>"
            f"<style>{_CSS}</style></head><body><nav>{nav}</nav><h1>{html.escape(title)}</h1>"
            f"<p>{html.escape(source)} · {html.escape(date)}</p>{body}</body></html>\n")


def _table(header: list[str], rows: list[list[str]], limit: int = 500, row_style=None, link_col=None) -> str:
    out = ["<table><tr>" + "".join(f"<th>{html.escape(h)}</th>" for h in header) + "</tr>"]
    for i, r in enumerate(rows[:limit]):
        st = f' style="background:{row_style(r)}"' if row_style else ""
        cells = []
        for j, c in enumerate(r):
            t = html.escape(c)
            if link_col and j in link_col and link_col[j](r):
                t = f'<a href="{html.escape(link_col[j](r))}">{t}</a>'
            cells.append(f"<td>{t}</td>")
        out.append(f"<tr{st}>" + "".join(cells) + "</tr>")
    return "\n".join(out) + "</table>"


def bar_chart(values: list[tuple], w: int = 640, h: int = 160, label: str = "") -> str:
    """Inline SVG bar chart of (x label, value) pairs."""
    if not values:
        return "<p>(no data)</p>"
    vmax = max(max(float(v) for _, v in values), 1.0)
    bw = w / len(values)
    bars = []
    for i, (x, v) in enumerate(values):
        bh = (h - 20) * float(v) / vmax
        bars.append(f'<rect class="bar" x="{i * bw + 1:.1f}" y="{h - 15 - bh:.1f}" width="{max(bw - 2, 1):.1f}" '
                    f'height="{bh:.1f}"><title>{html.escape(str(x))}: {v}</title></rect>')
        if len(values) <= 48:
            bars.append(f'<text class="axis" x="{i * bw + bw / 2:.1f}" y="{h - 3}" text-anchor="middle">'
                        f'{html.escape(str(x))}</text>')
    return (f'<svg width="{w}" height="{h}" role="img" aria-label="{html.escape(label)}">' + "".join(bars) + "</svg>")


def chord_svg(center: str, peers: list[tuple[str, float]], size: int = 360) -> str:
    """Radial chord view: the investigated IP in the middle, its peers on a circle, link width ∝
    bytes exchanged (the reference's chord diagram)."""
    if not peers:
        return "<p>(no peers)</p>"
    c = size / 2
    rad = c - 60
    vmax = max(max(v for _, v in peers), 1.0)
    parts = []
    for i, (p, v) in enumerate(peers):
        a = 2 * math.pi * i / len(peers)
        x, y = c + rad * math.cos(a), c + rad * math.sin(a)
        sw = 0.5 + 8.0 * math.sqrt(v / vmax)
        parts.append(f'<line x1="{c}" y1="{c}" x2="{x:.1f}" y2="{y:.1f}" stroke="#4a78b0" stroke-width="{sw:.1f}" '
                     f'stroke-opacity="0.6"><title>{html.escape(p)}: {int(v)} bytes</title></line>')
        parts.append(f'<text class="axis" x="{x:.1f}" y="{y:.1f}" text-anchor="middle">{html.escape(p)}</text>')
    parts.append(f'<circle cx="{c}" cy="{c}" r="6" fill="#b04a4a"/><text x="{c}" y="{c - 10}" '
                 f'text-anchor="middle" font-size="11">{html.escape(center)}</text>')
    return f'<svg width="{size}" height="{size}">' + "".join(parts) + "</svg>"


def load_threats(path: str) -> list[dict]:
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return json.load(f)


def add_threat(path: str, ip: str, title: str, comment: str, sev: int = 1) -> list[dict]:
    """Append/replace the analyst's storyboard entry for one IP (the reference's threat
    investigation "save" action)."""
    th = [t for t in load_threats(path) if t["ip"] != ip]
    th.append({"ip": ip, "title": title, "comment": comment, "sev": int(sev)})
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path + ".tmp", "w") as f:
        json.dump(th, f, indent=1)
    os.replace(path + ".tmp", path)
    return th


def render_all(source: str, date: str, day_dir: str, out_dir: str | None = None, limit: int = 500) -> list[str]:
    """Write suspicious.html, threat-<ip>.html (one per IP with details), storyboard.html and
    ingest_summary.html for a day. Returns the written paths."""
    out_dir = out_dir or os.path.join(day_dir, "ui")
    os.makedirs(out_dir, exist_ok=True)
    det = os.path.join(day_dir, "details")
    index = {}
    if os.path.exists(os.path.join(det, "index.json")):
        with open(os.path.join(det, "index.json")) as f:
            index = json.load(f)
    ips = index.get("ips", {})
    written = []
    # suspicious connects
    scores = os.path.join(day_dir, f"{source}_scores.csv")
    header, rows = [], []
    if os.path.exists(scores):
        with open(scores, newline="") as f:
            r = list(csv.reader(f))
        header, rows = (r[0], r[1:]) if r else ([], [])
    ipcols = [header.index(c) for c in ("srcIP", "dstIP", "ip_dst", "clientip") if c in header]
    links = {j: (lambda row, j=j: ips[row[j]].get("page", f"threat-{row[j]}.html") if row[j] in ips else None)
             for j in ipcols}
    body = _table(header, rows, limit, row_style=lambda row: SEV_COLORS.get(row[0], "#fff"), link_col=links)
    p = os.path.join(out_dir, "suspicious.html")
    with open(p, "w") as f:
        f.write(_page(f"Suspicious {source} connects", body, source, date))
    written.append(p)
    # threat investigation pages
    threats = {t["ip"]: t for t in load_threats(os.path.join(day_dir, "threats.json"))}
    for ip, ent in ips.items():
        parts = []
        if ip in threats:
            t = threats[ip]
            parts.append(f"<h2>{html.escape(t['title'])}</h2><p>{html.escape(t['comment'])}</p>")
        _, tl = _read_tsv(os.path.join(det, ent["timeline"]))
        parts.append("<h2>Timeline (events per hour)</h2>" + bar_chart([(int(a) % 86400 // 3600, int(b)) for a, b in tl],
                                                                         label="timeline"))
        if "chord" in ent:
            hd, ch = _read_tsv(os.path.join(det, ent["chord"]))
            parts.append("<h2>Peers (bytes)</h2>" + chord_svg(ip, [(r[1], float(r[2])) for r in ch[:24]]) + _table(hd, ch))
        if "dendro" in ent:
            hd, dd = _read_tsv(os.path.join(det, ent["dendro"]))
            parts.append("<h2>Queried domains</h2>" + _table(hd, dd))
        for row in index.get("rows", []):
            if row["ip"] == ip or row["peer"] == ip:
                hd, ed = _read_tsv(os.path.join(det, row["edge"]))
                parts.append(f"<h2>Edge {html.escape(row['ip'])} ↔ {html.escape(row['peer'])} hour {row['hour']:02d} "
                             f"(score {html.escape(row['score'])})</h2>" + _table(hd, ed, 200))
        p = os.path.join(out_dir, ent.get("page", f"threat-{ip}.html"))
        with open(p, "w") as f:
            f.write(_page(f"Threat investigation {ip}", "".join(parts), source, date))
        written.append(p)
    # storyboard
    sb = "".join(f"<h2><a href='{html.escape(ips.get(t['ip'], {}).get('page', 'threat-' + t['ip'] + '.html'))}'>{html.escape(t['title'])}</a> "
                 f"({html.escape(t['ip'])}, sev {t['sev']})</h2><p>{html.escape(t['comment'])}</p>"
                 for t in threats.values()) or "<p>No threats recorded (oni-oa threat ...).</p>"
    p = os.path.join(out_dir, "storyboard.html")
    with open(p, "w") as f:
        f.write(_page("Storyboard", sb, source, date))
    written.append(p)
    # ingest summary
    _, summ = _read_tsv(os.path.join(det, index.get("ingest_summary", "ingest_summary.tsv")))
    p = os.path.join(out_dir, "ingest_summary.html")
    with open(p, "w") as f:
        f.write(_page("Ingest summary", bar_chart([(int(a), int(b)) for a, b in summ], label="events per hour")
                      + _table(["hour", "events"], summ), source, date))
    written.append(p)
    return written
