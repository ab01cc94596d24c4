#!/usr/bin/env python3
"""Where does the word-sparse sampler (k_gibbs_ws) spend its steps? Runs a bench-size day's corpus
on the dense sampler and, at a few points of the chain, one diagnostic ws sweep with the kernel's
counters on: share of draws answered by the smoothing bucket, share of tokens whose word list
exceeds the register capacity, and the mean of the per-wave-step longest list.

  python tools/ws_probe.py --topics 100 [--flows 12500000] [--wide]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch

    from oni355 import ops
    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    from oni355.pipeline import common, flow
    from oni355.synth.flow import generate_flows

    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=12_500_000)
    ap.add_argument("--topics", type=int, default=100)
    ap.add_argument("--at", default="1,10,30,60,100,200")
    ap.add_argument("--wide", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    day = generate_flows(a.flows, seed=7, n_hosts=max(64, a.flows // 25), wide_vocab=a.wide)
    d = flow.to_device(day.cols, dev)
    cuts = flow.compute_cuts(d, None)
    sw, dw = flow.wordify(d, cuts)
    dk = ops.widen_pair(d["sip"], d["dip"])
    wk = ops.widen_pair(sw, dw)
    vocab = common.global_vocab(wk, None)
    run = common.build_and_train(dk, wk, None, vocab, a.topics, None, 0.01, 0x0D15EA5E, 0, 0, None, train=False)
    m = GibbsLDA(run.corpus, GibbsConfig(K=a.topics, sampler="ws", count_mode="auto"))
    m.initialize()
    stats = torch.zeros(5, dtype=torch.int64, device=dev)
    m._ws_tabs["stats"] = None
    done = 0
    for at in [int(x) for x in a.at.split(",")]:
        if at - 1 > done:
            m.sweep(at - 1 - done)
            done = at - 1
        stats.zero_()
        m._ws_tabs["stats"] = stats
        m.cfg.use_graph = False
        m._graph = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.sweep(1)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        m._ws_tabs["stats"] = None
        done += 1
        s = stats.cpu().tolist()
        print(json.dumps({"sweep": at, "tokens": s[0], "smoothing_frac": s[1] / max(s[0], 1),
                          "slow_list_frac": s[2] / max(s[0], 1), "sweep_ms_eager_with_counters": round(dt, 3),
                          "mean_wave_step_list_max": s[3] / max(s[4], 1), "lanes_per_step": s[0] / max(s[4], 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
