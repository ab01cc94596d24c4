#!/usr/bin/env python3
"""The analyst feedback loop ("noise filter", reference README.md:45-48)
on the realistic-vocabulary flow day, through the product's files:

  1. oni-ml day: the realistic day (bench.py --realistic-vocab: 12.5M flows, V ~ 1.7e5) → top-N
     results CSV (``<lpath>/flow/<date>/flow_results.csv``);
  2. ``oni-oa -d DATE -t flow`` enriches it into ``flow_scores.csv`` (sev = 0);
  3. the simulated analyst reviews the list and marks its false positives benign: every result row
     that is not a planted anomaly gets ``oni-oa score --rows … --sev 3`` (``--review N``: only the
     first N rows are reviewed);
  4. ``oni-oa publish`` copies the scores to ``<lpath>/flow_scores.csv`` -- what the next oni-ml run
     reads as feedback (sev = 3 rows × DUPFACTOR tokens on their IP documents);
  5. the same day again with that feedback.

Reports the planted recall before / after, how many marked rows were one-off rows of tiny hosts
(≤ --tiny flows in the day), and where the marked rows land in the second ranking.

  python tools/noise_filter_realistic.py --flows 12500000 > profiles/r5/noise_filter_realistic.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=12_500_000)
    ap.add_argument("--maxresults", type=int, default=3000)
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--review", type=int, default=0, help="rows the analyst reviews (0: all results)")
    ap.add_argument("--dupfactor", type=int, default=1000)
    ap.add_argument("--tiny", type=int, default=6, help="flows in the day of a 'tiny' host")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--lt-codebook", type=float, default=0.01)
    a = ap.parse_args()
    import torch

    from oni355 import schema
    from oni355.cli import oa
    from oni355.io import results as rio
    from oni355.oa import feedback as fbm
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows

    date = "20160708"
    lp = tempfile.mkdtemp(prefix="oni_noise_")
    t0 = time.perf_counter()
    day = generate_flows(a.flows, seed=7, n_hosts=max(64, a.flows // 25), wide_vocab=True, lt_codebook=a.lt_codebook)
    planted = np.asarray(day.anomaly_rows, dtype=np.int64)
    sip = np.asarray(day.cols["sip"])
    dip = np.asarray(day.cols["dip"])
    ips, cnt = np.unique(np.concatenate([sip, dip]), return_counts=True)

    def flows_of(ip):
        return cnt[np.searchsorted(ips, ip)]

    dev = torch.device(a.device)
    kw = dict(K=20, sweeps=a.sweeps, tol=1.0, maxresults=a.maxresults, device=dev, dupfactor=a.dupfactor)

    def one_run(feedback):
        ts = time.perf_counter()
        res = run_flow(day.cols, feedback=feedback, **kw)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        el = time.perf_counter() - ts
        rows = np.asarray(res.rows[: a.maxresults], dtype=np.int64)
        return res, rows, el

    res1, rows1, t1 = one_run(None)
    res_csv = os.path.join(lp, "flow", date, "flow_results.csv")
    rio.write_rendered(res_csv, schema.result_columns("flow"), rio.render_result("flow", day.cols, res1, 0))
    assert oa.main(["-d", date, "-t", "flow", "--lpath", lp, "--config", os.path.join(lp, "none.conf")]) == 0
    review = rows1 if a.review <= 0 else rows1[: a.review]
    fp_idx = [i for i, r in enumerate(review) if r not in set(planted.tolist())]
    fp_rows = review[fp_idx]
    assert oa.main(["score", "-d", date, "-t", "flow", "--lpath", lp, "--config", os.path.join(lp, "none.conf"),
                    "--rows", ",".join(map(str, fp_idx)), "--sev", "3"]) == 0
    assert oa.main(["publish", "-d", date, "-t", "flow", "--lpath", lp, "--config", os.path.join(lp, "none.conf")]) == 0
    fb = fbm.load_feedback(rio.scores_path(lp, "flow"), "flow")
    n_fb = len(fb["sip"]) if fb else 0
    res2, rows2, t2 = one_run(fb)
    pos2 = {int(r): i for i, r in enumerate(rows2)}
    still = [pos2[int(r)] for r in fp_rows if int(r) in pos2]
    tiny = np.minimum(flows_of(sip[fp_rows]), flows_of(dip[fp_rows])) <= a.tiny
    out = {
        "flows": a.flows, "vocab": int(res1.lda.vocab.numel()), "maxresults": a.maxresults,
        "planted": int(planted.size),
        "recall_before": round(float(np.isin(planted, rows1).mean()), 4),
        "recall_after": round(float(np.isin(planted, rows2).mean()), 4),
        "reviewed_rows": int(review.size), "marked_sev3": int(fp_rows.size), "feedback_rows_loaded": n_fb,
        "marked_tiny_host_rows": int(tiny.sum()),
        "marked_still_in_topN": len(still),
        "marked_still_in_topN_median_rank": (int(np.median(still)) + 1) if still else None,
        "day_s": [round(t1, 3), round(t2, 3)], "dupfactor": a.dupfactor, "sweeps": a.sweeps,
        "total_s": round(time.perf_counter() - t0, 1),
        "path": "results CSV -> oni-oa enrich -> oni-oa score --sev 3 -> oni-oa publish -> oni-ml feedback",
    }
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
