"""``oni-oa`` -- operational analytics (``start_oa.py -d YYYYMMDD -t TYPE -l LIMIT`` equivalent,
SURVEY.md §2.2 C27/C33, §3.5).

  oni-oa -d 20160708 -t flow -l 3000             # enrich results → <LPATH>/flow/20160708/flow_scores.csv
  oni-oa score -d 20160708 -t flow --ip 10.0.0.5 --sev 3    # analyst verdict
  oni-oa publish -d 20160708 -t flow             # copy day scores → <LPATH>/flow_scores.csv (ML feedback)
  oni-oa details -d 20160708 -t flow -l 10        # edge/chord/dendro/timeline TSVs of the top rows
  oni-oa threat -d 20160708 -t flow --ip 10.0.0.5 --title T --comment C   # storyboard entry
  oni-oa report -d 20160708 -t flow              # static pages: suspicious / threat-<ip> /
                                                 # storyboard / ingest_summary (<day>/ui/*.html)
"""
from __future__ import annotations

import argparse
import html
import os
import shutil
import sys


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = "enrich"
    if argv and argv[0] in ("enrich", "score", "publish", "report", "details", "threat"):
        cmd = argv.pop(0)
    ap = argparse.ArgumentParser(prog=f"oni-oa {cmd}")
    ap.add_argument("-d", "--date", required=True)
    ap.add_argument("-t", "--type", required=True, choices=["flow", "dns", "proxy"])
    ap.add_argument("-l", "--limit", type=int, default=None)
    ap.add_argument("--config", default=os.environ.get("ONI_CONFIG", "/etc/duxbay.conf"))
    ap.add_argument("--lpath", default=None)
    ap.add_argument("--iploc", default=None)
    ap.add_argument("--network-context", default=None)
    ap.add_argument("--reputation", default=None, help="e.g. csv:/path/indicators.csv")
    ap.add_argument("--ip", default=None)
    ap.add_argument("--word", default=None)
    ap.add_argument("--rows", default=None, help="comma-separated row indices")
    ap.add_argument("--sev", type=int, default=None)
    ap.add_argument("--html", default=None, help="report: also write the plain scores table here")
    ap.add_argument("--data-root", default=None, help="details: columnar store with the day's raw events")
    ap.add_argument("--input", action="append", default=[], help="details: raw input files instead of the store")
    ap.add_argument("--title", default="")
    ap.add_argument("--comment", default="")
    a = ap.parse_args(argv)
    from ..config import load_config
    from ..oa import enrich as en
    from ..oa import feedback as fb
    from ..oa.reputation import load_services
    cfg = load_config(a.config if os.path.exists(a.config) else None, LPATH=a.lpath,
                      IPLOC=a.iploc, NETWORK_CONTEXT=a.network_context)
    res_csv, scores_csv = en.default_paths(cfg.LPATH, a.type, a.date)
    if cmd == "enrich":
        geo = en.RangeTable.from_csv(cfg.IPLOC) if cfg.IPLOC else None
        ctx = en.RangeTable.from_csv(cfg.NETWORK_CONTEXT) if cfg.NETWORK_CONTEXT else None
        n = en.enrich(a.type, res_csv, scores_csv, a.limit, geo, ctx, load_services(a.reputation))
        print(f"{n} rows -> {scores_csv}")
        return 0
    if cmd == "score":
        if a.sev is None:
            ap.error("--sev is required")
        rows = [int(x) for x in a.rows.split(",")] if a.rows else None
        n = fb.set_severity(scores_csv, a.sev, ip=a.ip, word=a.word, rows=rows)
        print(f"{n} rows set to sev={a.sev} in {scores_csv}")
        return 0
    if cmd == "publish":
        from ..io import results as rio
        dst = rio.scores_path(cfg.LPATH, a.type)
        shutil.copyfile(scores_csv, dst)
        print(f"{scores_csv} -> {dst}")
        return 0
    day = os.path.dirname(scores_csv)
    if cmd == "details":
        from ..oa import details as det
        cols = _day_columns(a, cfg)
        idx = det.write_details(a.type, res_csv, cols, os.path.join(day, "details"), a.limit or 10)
        print(f"{len(idx['rows'])} rows, {len(idx['ips'])} IPs -> {os.path.join(day, 'details')}")
        return 0
    from ..oa import pages
    if cmd == "threat":
        if not a.ip:
            ap.error("--ip is required")
        th = pages.add_threat(os.path.join(day, "threats.json"), a.ip, a.title or f"Threat {a.ip}", a.comment,
                              a.sev if a.sev is not None else 1)
        print(f"{len(th)} threats in {os.path.join(day, 'threats.json')}")
        return 0
    written = pages.render_all(a.type, a.date, day, limit=a.limit or 500)
    print("\n".join(written))
    if not a.html:
        return 0
    from ..io import results as rio
    header, rows = rio.read_csv(scores_csv)
    out = a.html
    with open(out, "w") as f:
        f.write(f"<html><head><title>ONI {a.type} {a.date}</title></head><body><h1>{a.type} suspicious "
                f"connects {a.date}</h1><table border=1><tr>")
        f.write("".join(f"<th>{html.escape(h)}</th>" for h in header) + "</tr>\n")
        for r in rows[: a.limit or len(rows)]:
            f.write("<tr>" + "".join(f"<td>{html.escape(c)}</td>" for c in r) + "</tr>\n")
        f.write("</table></body></html>\n")
    print(out)
    return 0


def _day_columns(a, cfg) -> dict:
    """The day's raw events for the detail queries: decoded ``--input`` files, else the store."""
    if a.input:
        from .ml import _concat, _expand
        from ..io import decoders
        parts = []
        for f in _expand(a.input):
            if a.type == "flow":
                if f.endswith((".csv", ".txt")):
                    parts.append(decoders.read_flow_csv(f)[0])
                else:
                    from ..io import nfcapd
                    parts.append(nfcapd.read_nfcapd(f))
            elif a.type == "dns":
                parts.append(decoders.read_pcap_dns(f))
            else:
                parts.append(decoders.read_proxy_log(f))
        return _concat(parts)
    from ..store import columnar
    return columnar.read_day(a.data_root or cfg.DATA_ROOT, a.type, a.date)


if __name__ == "__main__":
    sys.exit(main())
