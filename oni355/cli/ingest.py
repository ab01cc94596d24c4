"""``oni-ingest`` -- collector + parallel decode workers into the columnar day store.

  oni-ingest -t flow --collector-path /data/nfcapd --data-root ./oni_store [--once] [--workers 8]
  oni-ingest -t dns --config ingest_conf.json            (reference ingest_conf.json layout)
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="oni-ingest")
    ap.add_argument("-t", "--type", required=True, choices=["flow", "dns", "proxy"])
    ap.add_argument("--collector-path", default=None)
    ap.add_argument("--data-root", default=None)
    ap.add_argument("--config", default=None, help="ingest_conf.json (pipelines.<type>.collector_path ...)")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--interval", type=float, default=5.0)
    ap.add_argument("--once", action="store_true")
    ap.add_argument("--move-to", default=None)
    a = ap.parse_args(argv)
    from ..ingest.watch import Collector
    collector_path, patterns, root = a.collector_path, None, a.data_root
    if a.config:
        with open(a.config) as f:
            conf = json.load(f)
        pipe = conf.get("pipelines", {}).get(a.type, {})
        collector_path = collector_path or pipe.get("collector_path")
        sf = pipe.get("supported_files")
        patterns = [sf] if isinstance(sf, str) else sf
        root = root or conf.get("data_root") or conf.get("hdfs_app_path")
    if not collector_path:
        ap.error("--collector-path (or --config) required")
    root = root or os.environ.get("ONI_DATA_ROOT", "./oni_store")
    c = Collector(a.type, collector_path, root, patterns, a.workers, a.move_to)
    if a.once:
        c.run_once()
    else:
        try:
            c.watch(a.interval)
        except KeyboardInterrupt:
            pass
    print(json.dumps(c.stats))
    return 0 if c.stats["errors"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
