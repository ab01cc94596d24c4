#!/usr/bin/env python3
"""Per-sweep time + topic-change fraction along the chain (sweeps 1..N after init) for each
count mode / sampler, on the bench corpus. Shows where each n_wk bookkeeping mode wins.

  python bench/gibbs_traj.py --flows 12500000 --sweeps 60 --modes recount,dual,recount+lds,dual+lds
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
    ap.add_argument("--sweeps", type=int, default=60)
    ap.add_argument("--modes", default="recount,dual,recount+lds,dual+lds")
    ap.add_argument("--chunk-len", type=int, default=0, help="0 = auto (global token count)")
    a = ap.parse_args()
    import torch

    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    from oni355.pipeline import common, flow
    from oni355.synth.flow import generate_flows

    dev = torch.device("cuda:0")
    day = generate_flows(a.flows, seed=7, n_hosts=max(64, a.flows // 25))
    d = flow.to_device(day.cols, dev)
    cuts = flow.compute_cuts(d, None)
    sw, dw = flow.wordify(d, cuts)
    dk = torch.cat([common.u32_to_i64(d["sip"]), common.u32_to_i64(d["dip"])])
    wk = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
    vocab = common.global_vocab(wk, None)
    run = common.build_and_train(dk, wk, None, vocab, a.topics, None, 0.01, 0x0D15EA5E, 0, a.chunk_len, None,
                                 train=False)
    c = run.corpus
    for mname in a.modes.split(","):
        m = GibbsLDA(c, GibbsConfig(K=a.topics, count_mode=mname.split("+")[0], use_graph=False,
                                    sampler=mname.split("+")[1] if "+" in mname else "auto"))
        m.initialize()
        torch.cuda.synchronize()
        ms, chg = [], []
        for _ in range(a.sweeps):
            z0 = m.tok_z.clone()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            m.sweep(1)
            ev[1].record()
            torch.cuda.synchronize()
            ms.append(round(ev[0].elapsed_time(ev[1]), 4))
            chg.append(round(float((m.tok_z != z0).sum()) / c.T, 4))
        print(json.dumps({"mode": mname, "ms": ms, "changed": chg, "mean_ms_11_60": sum(ms[10:60]) / max(len(ms[10:60]), 1)}),
              flush=True)
        del m
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
