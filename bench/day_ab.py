#!/usr/bin/env python3
"""Interleaved A/B of whole flow days on ONE generated day (one process: the 60 s generation of a
config-5 share is paid once, every variant runs the same events in alternation).

  python bench/day_ab.py --flows 62500000 --topics 100 --realistic-vocab --rounds 3 \\
      --variant base: --variant occ4:ONI_SAMPLER_AB=16 --variant L64:chunk=64

A variant is NAME:KEY=VALUE,... -- ONI_* keys are set in the environment for its days (read at
graph capture, so every day captures its own graphs), ``chunk`` is the chunk length (0 = auto).
Prints one JSON line per day and a summary (median / min ms per day and per training sweep).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_variant(s: str) -> tuple[str, dict, int]:
    name, _, rest = s.partition(":")
    env, chunk = {}, 0
    for kv in filter(None, rest.split(",")):
        k, _, v = kv.partition("=")
        if k == "chunk":
            chunk = int(v)
        elif k.startswith("ONI_"):
            env[k] = v
        else:
            raise SystemExit(f"variant {name}: only ONI_* keys and chunk=, got {k}")
    return name, env, chunk


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=12_500_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--realistic-vocab", action="store_true")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    import torch

    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows

    variants = [parse_variant(v) for v in a.variant]
    dev = torch.device(a.device)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    day = generate_flows(a.flows, seed=a.seed, n_hosts=max(64, a.flows // 25), wide_vocab=a.realistic_vocab)
    print(f"generated {a.flows} flows in {time.perf_counter() - t0:.1f} s", flush=True)
    base_env = dict(os.environ)
    res_by = {n: [] for n, _, _ in variants}
    # one untimed day first (module loads, allocator warm-up)
    run_flow(day.cols, K=a.topics, sweeps=a.sweeps, tol=1.0, maxresults=3000, device=dev)
    for r in range(a.rounds):
        for name, env, chunk in variants:
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(env)
            sync()
            ts = time.perf_counter()
            res = run_flow(day.cols, K=a.topics, sweeps=a.sweeps, tol=1.0, maxresults=3000, device=dev,
                           chunk_len=chunk)
            sync()
            wall = time.perf_counter() - ts
            t = res.timings
            train = t.get("train_dev_s", t.get("train_s", 0.0))
            rec = float(torch.isin(torch.as_tensor(day.anomaly_rows), torch.as_tensor(res.rows)).float().mean())
            line = {"variant": name, "round": r, "day_ms": round(wall * 1e3, 2),
                    "ms_per_sweep": round(train / a.sweeps * 1e3, 4), "recall": round(rec, 4),
                    "loglik": res.lda.model.likelihoods[-1][1] if res.lda.model.likelihoods else None}
            res_by[name].append(line)
            print(json.dumps(line), flush=True)
            del res
    os.environ.clear()
    os.environ.update(base_env)
    summary = {n: {"day_ms_median": statistics.median(x["day_ms"] for x in v),
                   "day_ms_min": min(x["day_ms"] for x in v),
                   "ms_per_sweep_median": statistics.median(x["ms_per_sweep"] for x in v),
                   "ms_per_sweep_min": min(x["ms_per_sweep"] for x in v)} for n, v in res_by.items()}
    out = {"flows": a.flows, "topics": a.topics, "realistic_vocab": a.realistic_vocab, "sweeps": a.sweeps,
           "rounds": a.rounds, "variants": {n: {"env": e, "chunk": c} for n, e, c in variants},
           "summary": summary, "days": res_by}
    print(json.dumps({"summary": summary}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
