#!/usr/bin/env python3
"""The product CLI, timed: ``oni-ml`` over several stored days (one process, the day pipeline of
oni355.pipeline.daily) and a cold single-day run (a fresh process: imports, HIP init, kernel
loading, graph capture -- what one ``ml_ops.sh YYYYMMDD flow`` costs).

  python bench/cli_days.py --flows 12500000 --days 5 --cold-flows 1000000

Writes the synthetic days into a columnar store first (not timed), then runs the CLI as child
processes and prints one JSON line: per-day seconds from the run's metrics.jsonl, the process wall
time of the multi-day run, and the cold config-2 (1M flows) wall time."""
from __future__ import annotations

import argparse
import datetime as dt
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=12_500_000)
    ap.add_argument("--days", type=int, default=5)
    ap.add_argument("--cold-flows", type=int, default=1_000_000)
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    from oni355.store import columnar
    from oni355.synth.flow import generate_flows

    tmp = tempfile.mkdtemp(prefix="oni_cli_days_")
    root, lp = os.path.join(tmp, "store"), os.path.join(tmp, "lp")
    d0 = dt.date(2016, 7, 8)
    dates = [(d0 + dt.timedelta(days=i)).strftime("%Y%m%d") for i in range(a.days)]
    t0 = time.perf_counter()
    for i, d in enumerate(dates):
        day = generate_flows(a.flows, seed=30 + i, n_hosts=max(64, a.flows // 25))
        columnar.write_day(root, "flow", d, day.cols)
        del day
        print(f"[cli_days] stored {d} at {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    conf = os.path.join(tmp, "none.conf")
    base = [sys.executable, "-m", "oni355.cli.ml"]
    common = ["flow", "1.0", "3000", "--data-root", root, "--lpath", lp, "--config", conf, "--device", a.device,
              "--sweeps", str(a.sweeps)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    t1 = time.perf_counter()
    r = subprocess.run(base + [f"{dates[0]}-{dates[-1]}", *common], capture_output=True, text=True, env=env,
                       timeout=1500, cwd=ROOT)
    multi_wall = time.perf_counter() - t1
    if r.returncode != 0:
        print(r.stderr[-3000:], file=sys.stderr)
        return 1
    per_day = []
    for d in dates:
        recs = [json.loads(x) for x in open(os.path.join(lp, "flow", d, "metrics.jsonl"))]
        per_day.append({k: recs[-1].get(k) for k in ("date", "day_s", "load_s", "loader_wait_s", "train_dev_s",
                                                      "h2d_copy_dev_s", "events")})
    # cold single day, config 2 (1M flows): a fresh process end to end
    cold_date = "20160801"
    day = generate_flows(a.cold_flows, seed=99, n_hosts=max(64, a.cold_flows // 25))
    columnar.write_day(root, "flow", cold_date, day.cols)
    t2 = time.perf_counter()
    r2 = subprocess.run(base + [cold_date, *common, "--quiet"], capture_output=True, text=True, env=env, timeout=900,
                        cwd=ROOT)
    cold_wall = time.perf_counter() - t2
    if r2.returncode != 0:
        print(r2.stderr[-3000:], file=sys.stderr)
        return 1
    cold_rec = [json.loads(x) for x in open(os.path.join(lp, "flow", cold_date, "metrics.jsonl"))][-1]
    steady = [p["day_s"] for p in per_day[1:]] or [per_day[0]["day_s"]]
    out = {"what": "oni-ml CLI over stored days (one process, day pipeline) + a cold single-day run",
           "flows_per_day": a.flows, "days": a.days, "sweeps": a.sweeps,
           "multi_day_process_wall_s": round(multi_wall, 3), "per_day": per_day,
           "steady_day_s_median": round(sorted(steady)[len(steady) // 2], 4),
           "cold_config2": {"flows": a.cold_flows, "process_wall_s": round(cold_wall, 3),
                            "in_process": {k: cold_rec.get(k) for k in ("load_s", "featurize_s", "vocab_s",
                                                                          "corpus_s", "init_s", "train_s",
                                                                          "score_s", "train_dev_s")}},
           "results_files": len(glob.glob(os.path.join(lp, "flow", "*", "flow_results.csv")))}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
