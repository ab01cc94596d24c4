#!/usr/bin/env python3
"""Log-likelihood and planted recall of whole flow days across Gibbs seeds, per sampler: is a gap
between two samplers' chains larger than the seed-to-seed spread of one?

  python tools/sampler_seed_spread.py --flows 12500000 --topics 100 --seeds 1,2,3 --samplers dense,mh
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=12_500_000)
    ap.add_argument("--topics", type=int, default=100)
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--samplers", default="dense,mh")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np

    from oni355.pipeline import flow
    from oni355.synth.flow import generate_flows
    day = generate_flows(a.flows, seed=7, n_hosts=max(64, a.flows // 25))
    res = {"flows": a.flows, "topics": a.topics, "sweeps": a.sweeps}
    for s in a.samplers.split(","):
        os.environ["ONI_SAMPLER"] = s
        rows = []
        for seed in [int(x) for x in a.seeds.split(",")]:
            r = flow.run_flow(day.cols, K=a.topics, sweeps=a.sweeps, maxresults=3000, seed=seed, device=a.device)
            rec = round(float(np.isin(day.anomaly_rows, np.asarray(r.rows)[:3000]).mean()), 4)
            rows.append({"seed": seed, "loglik": round(float(r.stats["loglik"]), 1), "recall": rec})
            print(json.dumps({"sampler": s, **rows[-1]}), flush=True)
        ll = np.array([x["loglik"] for x in rows])
        res[s] = {"runs": rows, "mean": float(ll.mean()), "spread_rel": float((ll.max() - ll.min()) / abs(ll.mean()))}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
