#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (sum over dispatches / dispatches).

usage: python tools/pmc_summary.py <dir-with-*counter_collection.csv> [--match REGEX] [--json out.json]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def load(d):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            rows += list(csv.DictReader(f))
    return rows


def summarise(rows, match=None):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in rows:
        k = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("Name")
        if match and not re.search(match, k or ""):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    out = {}
    for k, c in acc.items():
        n = max(len(disp[k]), 1)
        out[k] = {"dispatches": n, **{name: v / n for name, v in sorted(c.items())}}
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    merged = {}
    for d in a.dirs:
        for k, v in summarise(load(d), a.match).items():
            merged.setdefault(k, {}).update(v)
    for k, v in merged.items():
        print(k[:110])
        for name, val in v.items():
            print(f"    {name:28s} {val:16.1f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(merged, f, indent=1)
