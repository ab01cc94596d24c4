#!/usr/bin/env python3
"""Planted-anomaly recall of every source on default and realistic vocabularies, per anomaly
kind, at bench day sizes (one GPU). One JSON line per configuration (tools/recall_probe.py)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = [
    ("flow", 12_500_000, False, None), ("flow", 12_500_000, True, None),
    ("proxy", 2_000_000, False, "rare"), ("proxy", 2_000_000, False, "rare-active"),
    ("proxy", 2_000_000, True, "rare"), ("proxy", 2_000_000, True, "rare-active"),
    ("dns", 2_000_000, False, "rare"), ("dns", 2_000_000, True, "rare"), ("dns", 2_000_000, True, "rare-active"),
]

if __name__ == "__main__":
    only = sys.argv[1].replace("+", ",").split(",") if len(sys.argv) > 1 else None  # tools/gpu.sh splits at commas
    for src, n, wide, kind in CONFIGS:
        if only and src not in only:
            continue
        cmd = [sys.executable, os.path.join(ROOT, "tools", "recall_probe.py"), "--source", src, "--n", str(n)]
        if wide:
            cmd.append("--wide")
        if kind:
            cmd += ["--anomaly-kind", kind]
        print(json.dumps({"start": [src, n, wide, kind]}), file=sys.stderr, flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        print(line[-1] if line else json.dumps({"source": src, "wide": wide, "kind": kind, "error": r.stderr[-500:]}),
              flush=True)
