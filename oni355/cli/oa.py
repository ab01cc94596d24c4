"""``oni-oa`` -- operational analytics (``start_oa.py -d YYYYMMDD -t TYPE -l LIMIT`` equivalent,
SURVEY.md §2.2 C27/C33, §3.5).

  oni-oa -d 20160708 -t flow -l 3000             # enrich results → <LPATH>/flow/20160708/flow_scores.csv
  oni-oa score -d 20160708 -t flow --ip 10.0.0.5 --sev 3    # analyst verdict
  oni-oa publish -d 20160708 -t flow             # copy day scores → <LPATH>/flow_scores.csv (ML feedback)
  oni-oa report -d 20160708 -t flow --html out.html          # static HTML table of the scores
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
    if argv and argv[0] in ("enrich", "score", "publish", "report"):
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
    ap.add_argument("--html", default=None)
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
    from ..io import results as rio
    header, rows = rio.read_csv(scores_csv)
    out = a.html or scores_csv.replace(".csv", ".html")
    with open(out, "w") as f:
        f.write(f"<html><head><title>ONI {a.type} {a.date}</title></head><body><h1>{a.type} suspicious "
                f"connects {a.date}</h1><table border=1><tr>")
        f.write("".join(f"<th>{html.escape(h)}</th>" for h in header) + "</tr>\n")
        for r in rows[: a.limit or len(rows)]:
            f.write("<tr>" + "".join(f"<td>{html.escape(c)}</td>" for c in r) + "</tr>\n")
        f.write("</table></body></html>\n")
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
