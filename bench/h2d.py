#!/usr/bin/env python3
"""Host → HBM upload of one GPU's synthetic flow day: pinned staging ring vs plain ``.to()``.

Times ``flow.to_device`` (9 columns, 12.5M flows by default) both ways, then upload + the first
device stage (flow keys → quantile cuts) to show the copies overlapping host work. One JSON line.
  python bench/h2d.py [--flows 12500000] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=12_500_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    from oni355.io import staging
    from oni355.pipeline import flow
    from oni355.synth.flow import generate_flows

    dev = torch.device("cuda:0")
    day = generate_flows(a.flows, seed=7)
    nbytes = sum(flow.to_device({k: v[:1] for k, v in day.cols.items()}, "cpu")[k].element_size() * a.flows
                 for k in flow.DEVICE_COLS)

    def timed(m: str, with_cuts: bool) -> float:
        os.environ["ONI_STAGED_H2D"] = m
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            d = flow.to_device(day.cols, dev)
            if with_cuts:
                flow.compute_cuts(d, None)
            torch.cuda.synchronize(dev)
            best = min(best, time.perf_counter() - t0)
            del d
        return best

    modes = {"plain": "0", "ring": "1", "reg": "reg"}
    for m in modes.values():
        timed(m, True)  # warm every path (allocator, library load)
    r = {"flows": a.flows, "bytes": nbytes}
    for tag, m in modes.items():
        r[f"{tag}_upload_ms"] = round(timed(m, False) * 1e3, 2)
        r[f"{tag}_GBps"] = round(nbytes / (r[f"{tag}_upload_ms"] * 1e-3) / 1e9, 2)
        r[f"{tag}_upload_plus_cuts_ms"] = round(timed(m, True) * 1e3, 2)
    r["stage_chunk_MB"] = staging.CHUNK_BYTES >> 20
    r["stage_threads"] = staging.THREADS
    print(json.dumps(r))
    return 0


if __name__ == "__main__":
    sys.exit(main())
