#!/usr/bin/env python3
"""X01 payload of a W-rank day, measured on one GPU: generate the W weak-scaled shards (12.5M flows
each, the bench's per-GPU share; --wide = the realistic-vocabulary day), wordify each with shard 0's
cuts, take every word's maximum local token count over the shards, classify the words as the
sampler does (models/gibbs.py _setup_x01: tiny ≤ ⌊127/W⌋, light ≤ ⌊32767/W⌋, else heavy) and report
the packed vs dense per-sweep payload.

  python tools/x01_payload.py --wide --worlds 2,4,8
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
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--wide", action="store_true")
    ap.add_argument("--K", type=int, default=20)
    a = ap.parse_args()
    import torch

    from oni355 import ops
    from oni355.models.gibbs import NK_REP
    from oni355.pipeline import common, flow
    from oni355.synth.flow import generate_flows

    dev = torch.device("cuda:0")
    from oni355.models.gibbs import tiling_for
    G, KP = tiling_for(a.K)  # the tiling the model of K topics samples with (K ≥ 100: MH, KS = K)
    KS = G * KP
    a.worlds = a.worlds.replace("+", ",")  # tools/gpu.sh splits arguments at commas
    Wmax = max(int(w) for w in a.worlds.split(","))
    shard_words, cuts = [], None
    for r in range(Wmax):
        day = generate_flows(a.flows, seed=7, rank=r, wide_vocab=a.wide)
        d = flow.to_device(day.cols, dev)
        if cuts is None:
            cuts = flow.compute_cuts(d, None)
        else:
            flow.compute_cuts(d, None)  # keys for wordify; shard 0's cuts are used
        sw, dw = flow.wordify(d, cuts)
        wk = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
        u, c = torch.unique(wk, return_counts=True)
        shard_words.append((u, c))
        del d, day
    out = {"flows_per_rank": a.flows, "wide": a.wide, "K": a.K, "KS": KS, "worlds": {}}
    for W in (int(w) for w in a.worlds.split(",")):
        vocab = torch.unique(torch.cat([u for u, _ in shard_words[:W]]))
        mx = torch.zeros(vocab.numel(), dtype=torch.int64, device=dev)
        cg = torch.zeros(vocab.numel(), dtype=torch.int64, device=dev)
        for u, c in shard_words[:W]:
            idx = torch.searchsorted(vocab, u)
            mx[idx] = torch.maximum(mx[idx], c)
            cg[idx] += c
        O8, O = 127 // W, 32767 // W
        T = int((mx <= O8).sum())
        L = int(((mx > O8) & (mx <= O)).sum())
        H = int((mx > O).sum())
        tail = NK_REP * KS + ops.DN_AUX
        V = int(vocab.numel())
        packed = ops.x01_packed_len(T, L, H, KS, tail) * 4
        packed16 = ops.x01_packed_len(0, T + L, H, KS, tail) * 4
        dense = (V * KS + tail) * 4
        # modular classes (the sum taken mod 2^8 / 2^16 in int8 / int16 collectives): a word's
        # global value lies in [-c_w, c_w] for its GLOBAL count c_w, so the class depends on c_w
        # alone -- no per-rank offsets, no 1/W shrink of the ranges
        mT = int((cg <= 127).sum())
        mL = int(((cg > 127) & (cg <= 32767)).sum())
        mH = int((cg > 32767).sum())
        modular = (mT * KS + 2 * mL * KS + 4 * mH * KS + 4 * tail)
        out["worlds"][W] = dict(V=V, tiny=T, light=L, heavy=H, dense_MB=round(dense / 1e6, 3),
                                packed16_MB=round(packed16 / 1e6, 3), packed_MB=round(packed / 1e6, 3),
                                modular_tiny=mT, modular_light=mL, modular_heavy=mH,
                                modular_MB=round(modular / 1e6, 3))
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
