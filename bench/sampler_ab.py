#!/usr/bin/env python3
"""Interleaved A/B of sampler kernel variants on one corpus (one process, N variants x M rounds):
each variant is a (sampler, ONI_SAMPLER_AB) pair; every model burns in, then rounds time
``--sweeps`` sweeps of each variant in turn (graph-replayed, as in a day). Prints ms per sweep.

  python bench/sampler_ab.py --topics 20 --variants x1:0,x1:1,x1:2,generic:0
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
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--sweeps", type=int, default=20)
    ap.add_argument("--burn", type=int, default=150)
    ap.add_argument("--variants", default="x1:0,x1:1,x1:2,x1:3,generic:0")
    ap.add_argument("--count-mode", default="auto")
    ap.add_argument("--wide", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch

    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    from oni355.pipeline import common, flow
    from oni355.synth.flow import generate_flows

    dev = torch.device("cuda:0")
    day = generate_flows(a.flows, seed=7, n_hosts=max(64, a.flows // 25), wide_vocab=a.wide)
    d = flow.to_device(day.cols, dev)
    cuts = flow.compute_cuts(d, None)
    sw, dw = flow.wordify(d, cuts)
    dk = torch.cat([common.u32_to_i64(d["sip"]), common.u32_to_i64(d["dip"])])
    wk = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
    vocab = common.global_vocab(wk, None)
    run = common.build_and_train(dk, wk, None, vocab, a.topics, None, 0.01, 0x0D15EA5E, 0, 128, None, train=False)
    c = run.corpus
    variants = a.variants.split(",")
    models = {}
    for v in variants:
        sampler, var = v.split(":")
        os.environ["ONI_SAMPLER_AB"] = var
        m = GibbsLDA(c, GibbsConfig(K=a.topics, count_mode=a.count_mode, sampler=sampler))
        m.initialize()
        m.sweep(a.burn)
        models[v] = m
    torch.cuda.synchronize()
    times = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v, m in models.items():
            os.environ["ONI_SAMPLER_AB"] = v.split(":")[1]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            m.sweep(a.sweeps)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.sweeps)
    out = {v: {"ms_per_sweep_median": round(float(np.median(t)), 4), "min": round(float(np.min(t)), 4),
               "mode": m._sweep_mode(m.sweeps_done), "change_log_tail": m.change_log[-2:]}
           for (v, t), m in zip(times.items(), models.values())}
    print(json.dumps({"topics": a.topics, "tokens": int(c.T), "burn": a.burn, "variants": out}), flush=True)
    # identical chains: every variant draws the same topics
    ref = next(iter(models.values()))
    print(json.dumps({"bitwise_equal": all(torch.equal(ref.tok_z, m.tok_z) for m in models.values())}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
