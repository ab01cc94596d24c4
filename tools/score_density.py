#!/usr/bin/env python3
"""MFMA score-tile density study: block density of 16x16 (doc, word) tiles
under the default heaviest-first doc order and MinHash word-set orderings. CPU only.

  python tools/score_density.py [n_flows]
"""
import sys, time, numpy as np, torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from oni355.synth.flow import generate_flows
from oni355.pipeline import flow as F, common
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
day = generate_flows(n, seed=7, n_hosts=max(64, n // 25))
d = F.to_device(day.cols, "cpu"); cuts = F.compute_cuts(d, None); sw, dw = F.wordify(d, cuts)
dk = torch.cat([common.u32_to_i64(d["sip"]), common.u32_to_i64(d["dip"])])
wk = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
vocab, wids = common.encode_words(wk, None)
udoc, inv = common.encode_docs(dk)
D, V = udoc.numel(), vocab.numel()
u = torch.unique(inv.long() * V + wids.long())
pdoc, pword = u // V, u % V
plan, _ = common.tile_plan(pdoc, pword, D, V)
print("pairs", u.numel(), "docs", D, "V", V, "baseline density", round(plan.density(), 4), "items", plan.n_items)
# MinHash reorder: docs sorted by (minhash_1, minhash_2) of their word sets, then tile
def minhash(seed):
    h = (pword * (2 * seed + 0x9E3779B1) + seed * 0x85EBCA77) % 2147483647
    return torch.full((D,), 2**62, dtype=torch.int64).scatter_reduce_(0, pdoc, h, reduce="amin")
for nh in (1, 2, 4):
    keys = [minhash(s) for s in range(nh)]
    order = torch.arange(D)
    for k in reversed(keys):
        order = order[torch.sort(k[order], stable=True)[1]]
    rank = torch.empty(D, dtype=torch.int64); rank[order] = torch.arange(D)
    # relabel docs so tile_plan's heaviest-first ordering is replaced by the minhash order
    npairs = torch.bincount(pdoc, minlength=D)
    # tile_plan orders by (npairs desc, first word); emulate a pure minhash order by monkeypatching ranks:
    pd2 = rank[pdoc]
    # build tiles of 16 consecutive docs in minhash order, blocks of 16 distinct words per tile
    tile = pd2 // 16
    tw = torch.unique(tile * V + pword)
    tcount = torch.bincount(tw // V, minlength=(D + 15) // 16)
    items = int(((tcount + 15) // 16).sum())
    print("minhash", nh, "density", round(u.numel() / (256 * items), 4), "items", items)
# exact ceiling-ish: group docs by identical word sets (perfect overlap)
