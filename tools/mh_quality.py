#!/usr/bin/env python3
"""Chain quality of the MH sampler against the exact Gibbs chain (verdict r3 next-round item 2):
log-likelihood trajectory of both on one synthetic flow day, same seed, same K.

  python tools/mh_quality.py --flows 40000 --topics 100 --sweeps 200 [--device cuda]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def chain(a, sampler: str, cycles: int, z0=None, burn: int = 0, sweeps: int | None = None):
    """One chain; ``z0`` (canonical z after ``burn`` sweeps of another chain) starts it from that
    state: does the MH chain hold the dense chain's equilibrium, or drift off it?"""
    import torch

    from oni355.models.corpus import auto_chunk_len, build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA, tiling_for
    from oni355.pipeline import common, flow
    from oni355.synth.flow import generate_flows

    os.environ["ONI_MH_DOC_MOVES"] = str(cycles)
    dev = torch.device(a.device)
    day = generate_flows(a.flows, seed=7, n_hosts=max(64, a.flows // 25), wide_vocab=a.wide)
    d = flow.to_device(day.cols, dev)
    cuts = flow.compute_cuts(d, None)
    sw, dw = flow.wordify(d, cuts)
    dk = torch.cat([common.u32_to_i64(d["sip"]), common.u32_to_i64(d["dip"])])
    wk = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
    vocab = common.global_vocab(wk, None)
    udoc, inv = torch.unique(dk, return_inverse=True)
    wi = torch.searchsorted(vocab, wk).to(torch.int32)
    G, _ = tiling_for(a.topics, sampler)
    L = a.chunk_len or auto_chunk_len(int(dk.numel()), G, hi=127 if sampler == "mh" else 128)
    c = build_corpus(inv.to(torch.int32), wi, int(udoc.numel()), int(vocab.numel()), common.i64_to_u32bits(udoc), G, L)
    m = GibbsLDA(c, GibbsConfig(K=a.topics, sampler=sampler, post_samples=1, use_graph=a.device != "cpu"))
    if z0 is None:
        m.initialize()
    else:
        m.load_canonical_z(z0, burn)
        print(json.dumps({"sampler": sampler, "start": burn, "loglik": round(m.log_likelihood(), 2)}), flush=True)
    traj = []
    t0 = time.time()
    done = 0
    for stop in range(a.every, (sweeps or a.sweeps) + 1, a.every):
        m.sweep(stop - done)
        done = stop
        traj.append((burn + done, round(m.log_likelihood(), 2)))
        print(json.dumps({"sampler": sampler, "burn": burn, "cycles": cycles, "sweep": burn + done,
                          "loglik": traj[-1][1], "change": m.change_log[-1][1] if m.change_log else None,
                          "s": round(time.time() - t0, 1)}), flush=True)
    return {"L": L, "G": G, "T": int(c.T), "traj": traj}, m.canonical_z().cpu()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=40000)
    ap.add_argument("--topics", type=int, default=100)
    ap.add_argument("--sweeps", type=int, default=200)
    ap.add_argument("--every", type=int, default=20)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--chunk-len", type=int, default=0)
    ap.add_argument("--doc-moves", default="1,2")
    ap.add_argument("--wide", action="store_true")
    ap.add_argument("--skip-plain", action="store_true", help="no MH chain from the random start")
    ap.add_argument("--burn", default="", help="comma list: also run MH from the dense chain's state after this many sweeps")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = {"flows": a.flows, "topics": a.topics}
    res["gibbs"], _ = chain(a, "dense", 1)
    burns = [int(x) for x in a.burn.split(",") if x]
    zb = {b: chain(a, "dense", 1, sweeps=b)[1] for b in burns}
    for cy in [int(x) for x in a.doc_moves.split(",") if x]:
        if not a.skip_plain:
            res[f"mh{cy}"], _ = chain(a, "mh", cy)
        for b in burns:
            res[f"mh{cy}_after_burn{b}"], _ = chain(a, "mh", cy, zb[b], b, a.sweeps - b)
    g = res["gibbs"]["traj"][-1][1]
    for k in list(res):
        if k.startswith("mh"):
            res[k]["final_rel_to_gibbs"] = round((res[k]["traj"][-1][1] - g) / abs(g), 5)
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
