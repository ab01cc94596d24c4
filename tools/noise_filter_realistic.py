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
    ap.add_argument("--rounds", type=int, default=2,
                    help="feedback rounds: each reviews the latest top-N, marks its new false positives and "
                         "reruns the day with every verdict so far")
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

    cfgp = os.path.join(lp, "none.conf")
    planted_set = set(planted.tolist())

    def review(res, rows, rnd):
        """The analyst's pass over one day's results: enrich, mark the unplanted rows benign, publish."""
        res_csv = os.path.join(lp, "flow", date, "flow_results.csv")
        rio.write_rendered(res_csv, schema.result_columns("flow"), rio.render_result("flow", day.cols, res, 0))
        assert oa.main(["-d", date, "-t", "flow", "--lpath", lp, "--config", cfgp]) == 0
        seen = rows if a.review <= 0 else rows[: a.review]
        idx = [i for i, r in enumerate(seen) if int(r) not in planted_set]
        if idx:
            assert oa.main(["score", "-d", date, "-t", "flow", "--lpath", lp, "--config", cfgp,
                            "--rows", ",".join(map(str, idx)), "--sev", "3"]) == 0
        assert oa.main(["publish", "-d", date, "-t", "flow", "--lpath", lp, "--config", cfgp]) == 0
        return seen[idx], fbm.load_feedback(rio.scores_path(lp, "flow"), "flow")

    res, rows, t = one_run(None)
    rounds = [{"recall": round(float(np.isin(planted, rows).mean()), 4), "day_s": round(t, 3)}]
    fb_all, marked_all = None, np.zeros(0, np.int64)
    for rnd in range(a.rounds):
        marked, fb = review(res, rows, rnd)
        marked_all = np.concatenate([marked_all, marked])
        if fb is not None:
            # the analyst's verdicts accumulate over the rounds (each publish holds one day's review)
            fb_all = fb if fb_all is None else {k: (np.concatenate([fb_all[k], fb[k]]) if isinstance(fb[k], np.ndarray)
                                                    else fb[k]) for k in fb}
        res, rows, t = one_run(fb_all)
        pos = {int(r): i for i, r in enumerate(rows)}
        still = [pos[int(r)] for r in marked_all if int(r) in pos]
        tiny = np.minimum(flows_of(sip[marked]), flows_of(dip[marked])) <= a.tiny if marked.size else np.zeros(0, bool)
        rounds.append({"recall": round(float(np.isin(planted, rows).mean()), 4), "day_s": round(t, 3),
                       "marked_this_round": int(marked.size), "marked_tiny_host_rows": int(tiny.sum()),
                       "feedback_rows_total": int(len(fb_all["sip"])) if fb_all else 0,
                       "marked_still_in_topN": len(still),
                       "marked_still_in_topN_median_rank": (int(np.median(still)) + 1) if still else None})
    out = {
        "flows": a.flows, "vocab": int(res.lda.vocab.numel()), "maxresults": a.maxresults,
        "planted": int(planted.size), "recall_before": rounds[0]["recall"], "recall_after": rounds[-1]["recall"],
        "rounds": rounds, "reviewed_rows_per_round": a.review or a.maxresults, "dupfactor": a.dupfactor,
        "sweeps": a.sweeps, "total_s": round(time.perf_counter() - t0, 1),
        "path": "results CSV -> oni-oa enrich -> oni-oa score --sev 3 -> oni-oa publish -> oni-ml feedback",
    }
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
