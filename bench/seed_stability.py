#!/usr/bin/env python3
"""Seed stability of the top-N (verdict r3 item 4): the suspicious rows an analyst reviews should be
a property of the data, not of the sampler's seed. Runs the bench day (12.5M flows, K = 20, 200
sweeps, top-3000) with several LDA seeds on one GPU and reports the mean pairwise overlap of the
top-N row sets, planted recall per seed, and day time; the same for the realistic-vocabulary day.

  python bench/seed_stability.py --seeds 3
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=12_500_000)
    ap.add_argument("--seeds", type=int, default=3)
    ap.add_argument("--maxresults", type=int, default=3000)
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--days", default="default,realistic")
    ap.add_argument("--deep", type=int, default=4, help="also rank each seed's rows this many times deeper")
    ap.add_argument("--beta", type=float, default=0.01, help="LDA β (estimator A/B)")
    a = ap.parse_args()
    import numpy as np
    import torch

    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows

    out = {"flows": a.flows, "maxresults": a.maxresults, "sweeps": a.sweeps, "beta": a.beta, "post_samples":
           os.environ.get("ONI_POST_SAMPLES", "default"), "chains": int(os.environ.get("ONI_CHAINS", "1")), "days": {}}
    for kind in a.days.split(","):
        day = generate_flows(a.flows, seed=7, wide_vocab=kind == "realistic")
        planted = set(np.asarray(day.anomaly_rows).tolist())
        tops, rec, times = [], [], []
        run_flow(day.cols, K=20, sweeps=4, maxresults=10, device="cuda:0")  # warm-up (code objects, pools)
        for i in range(a.seeds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = run_flow(day.cols, K=20, sweeps=a.sweeps, maxresults=a.maxresults * a.deep, device="cuda:0",
                           seed=0x0D15EA5E + 7919 * i, beta=a.beta)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            deep = np.asarray(res.rows)
            tops.append((set(deep[: a.maxresults].tolist()), set(deep.tolist()), np.asarray(res.scores), deep))
            rows = tops[-1][0]
            rec.append(len(rows & planted) / max(len(planted), 1))
        ov = [len(x[0] & y[0]) / a.maxresults for x, y in itertools.combinations(tops, 2)]
        # boundary jitter: how much of one seed's top-N is inside another seed's top-(deep·N)
        ovd = [len(x[0] & y[1]) / a.maxresults for x, y in itertools.permutations(tops, 2)]
        # where do the rows that leave the top-N go, and how much does one row's score move between
        # seeds? (the cut falls in a smooth score density: rows near it trade places with the
        # posterior estimate's seed-to-seed noise, not with exact ties)
        anat = []
        for x, y in itertools.permutations(tops, 2):
            ry = {int(r): i for i, r in enumerate(y[3])}
            sy = y[2]
            lost = [int(r) for r in x[3][: a.maxresults] if int(r) not in y[0]]
            lost_rank = np.array([ry.get(r, len(y[3])) for r in lost]) + 1
            both = [(i, ry[int(r)]) for i, r in enumerate(x[3]) if int(r) in ry]
            lr = np.abs(np.log(np.array([x[2][i] / sy[j] for i, j in both])))
            near = [i for i, j in both if i < a.maxresults]
            lr_top = np.abs(np.log(np.array([x[2][i] / sy[ry[int(x[3][i])]] for i in near])))
            anat.append({"lost": len(lost), "lost_rank_in_other_median": int(np.median(lost_rank)) if lost else None,
                         "lost_rank_in_other_p90": int(np.percentile(lost_rank, 90)) if lost else None,
                         "lost_beyond_deep": int((lost_rank > len(y[3])).sum()),
                         "score_abs_log_ratio_median_topN": round(float(np.median(lr_top)), 4),
                         "score_abs_log_ratio_median_deep": round(float(np.median(lr)), 4)})
        sc = tops[0][2]
        # rank distance that the median seed-to-seed score change spans at the cut
        med = float(np.median([v["score_abs_log_ratio_median_topN"] for v in anat]))
        cut = sc[a.maxresults - 1]
        lo, hi = np.searchsorted(sc, cut * np.exp(-med)), np.searchsorted(sc, cut * np.exp(med))
        margin = {"score_at_N": float(sc[a.maxresults - 1]), "score_at_N_over_2": float(sc[a.maxresults // 2]),
                  "score_at_deep": float(sc[-1]), "rows_within_1pct_of_score_at_N":
                  int(((sc >= sc[a.maxresults - 1] * 0.99) & (sc <= sc[a.maxresults - 1] * 1.01)).sum())}
        out["days"][kind] = {"topN_overlap_mean": round(float(np.mean(ov)), 4), "topN_overlap_pairs": [round(v, 4) for v in ov],
                             f"topN_within_top{a.deep}N_mean": round(float(np.mean(ovd)), 4), "margin_seed0": margin,
                             "boundary_anatomy": anat,
                             "ranks_spanned_by_median_score_noise_at_N": [int(lo) + 1, int(hi) + 1],
                             "recall": [round(r, 4) for r in rec], "day_s": [round(t, 4) for t in times],
                             "vocab": int(res.stats.get("V", 0)), "loglik": float(res.stats["loglik"])}
        print(json.dumps({kind: out["days"][kind]}), file=sys.stderr, flush=True)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
