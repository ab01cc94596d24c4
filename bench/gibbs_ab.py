#!/usr/bin/env python3
"""Interleaved A/B of sampler count modes on one corpus (cdna guide §5.4 rule 24: one process,
N variants × M rounds). Prints per-variant median/min ms per sweep + per-stage event timings.

  python bench/gibbs_ab.py --flows 12500000 --rounds 5 --sweeps 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=12_500_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sweeps", type=int, default=20)
    ap.add_argument("--burn", type=int, default=30)
    ap.add_argument("--modes", default="delta,delta+qpf,recount,dual", help="count_mode[+sampler], separated by , or /")
    ap.add_argument("--chunk-len", type=int, default=128)
    ap.add_argument("--chunk-lens", default="", help="extra A/B: comma list of L values (dual+qpf)")
    ap.add_argument("--lds", action="store_true", help="chunk-length A/B with the LDS-count sampler")
    ap.add_argument("--wide", action="store_true", help="realistic-vocabulary flow day (synth.flow wide_vocab)")
    ap.add_argument("--lt-codebook", type=float, default=0.01, help="--wide: long-tail behaviours per flow")
    a = ap.parse_args()
    import numpy as np
    import torch

    from oni355 import ops
    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    from oni355.pipeline import common, flow
    from oni355.synth.flow import generate_flows

    dev = torch.device("cuda:0")
    day = generate_flows(a.flows, seed=7, n_hosts=max(64, a.flows // 25), wide_vocab=a.wide,
                         lt_codebook=a.lt_codebook)
    d = flow.to_device(day.cols, dev)
    cuts = flow.compute_cuts(d, None)
    sw, dw = flow.wordify(d, cuts)
    dk = torch.cat([common.u32_to_i64(d["sip"]), common.u32_to_i64(d["dip"])])
    wk = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
    vocab = common.global_vocab(wk, None)
    run = common.build_and_train(dk, wk, None, vocab, a.topics, None, 0.01, 0x0D15EA5E, 0, a.chunk_len, None,
                                 train=False)
    c = run.corpus
    print(json.dumps({"corpus": c.stats()}), flush=True)
    modes = a.modes.replace("/", ",").split(",")
    models = {m: GibbsLDA(c, GibbsConfig(K=a.topics, count_mode=m.split("+")[0],
                                         sampler=m.split("+")[1] if "+" in m else "auto"))
              for m in modes}
    for m in models.values():
        m.initialize()
        m.sweep(a.burn)
    torch.cuda.synchronize()
    # change rate at this point of the chain
    m0 = models[modes[0]]
    z0 = m0.tok_z.clone()
    m0.sweep(1)
    torch.cuda.synchronize()
    changed = float((m0.tok_z != z0).sum()) / c.T
    res = {m: [] for m in modes}
    for _ in range(a.rounds):
        for name, m in models.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.sweep(a.sweeps)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / a.sweeps * 1e3)
    out = {"changed_frac": changed, "T": c.T, "modes_at_stage_timing": {k: v._sweep_mode(v.sweeps_done + 1) for k, v in models.items()}}
    for name, v in res.items():
        out[name] = {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))}
    # per-stage timing (eager, events) for each mode
    for name, m in models.items():
        st = {}
        md = m._sweep_mode(m.sweeps_done + 1)
        for stage in range(5):
            if stage == 3 and md != 3:
                continue
            if stage == 4 and not m.mh:
                continue
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ts = []
            for _ in range(5):
                ev[0].record()
                head = m.dn[m.b][: m.V * m.KS].view(m.V, m.KS)
                if stage == 0:
                    st0 = m._state(False)
                    if m.mh:
                        st0.update(m.mh_state())
                    ops.gibbs_pass(st0, m.G, m.KP, m.K, m.alpha, m.cfg.seed, False, m.sweep_ctr,
                                   c.chunk_len, mode=md, sampler=m.qpf, alpha_in_row=m._air,
                                   mh_doc_moves=getattr(m, "mh_doc_moves", 1),
                                   chg_mask=m.wbits if md == 4 else getattr(m, "chg_mask", None), wpos=c.wpos,
                                   z_w=getattr(m, "z_w", None), zz_w=getattr(m, "zz_w", None))
                elif stage == 1 and md == 0:
                    ops.recount(c.wsorted, c.wslot, m.tok_z, head, m.KS)
                elif stage == 1 and md == 3:
                    ops.recount(c.wsorted, None, m.z_w, head, m.KS)
                elif stage == 1 and md == 4:
                    ops.wdelta_recount(m.wbits, c.wsorted, m.zz_w, head, m.KS)
                elif stage == 1 and md == 2:
                    ops.delta_recount(c.wslot, c.tile_wlo, c.tile_whi, m.chg_mask, c.tok_word, m.tok_z, m.tok_zprev,
                                      head, m.KS, m.G)
                elif stage == 3:
                    ops.STREAM_RECOUNT = not ops.STREAM_RECOUNT
                    ops.recount(c.wsorted, None, m.z_w, head, m.KS)
                    ops.STREAM_RECOUNT = not ops.STREAM_RECOUNT
                elif stage == 4:
                    m.mh_build_tables()
                elif stage == 2:
                    ops.gibbs_apply(m.nwk, m.dn[m.b], m.dn[1 - m.b], m.nk[m.cn], m.nk[1 - m.cn], m.q, m.qfix, m.V, m.K, m.KS,
                                    m.beta, m.vbeta, m.sweep_ctr, bump=False, absolute=md in (0, 3))
                ev[1].record()
                torch.cuda.synchronize()
                ts.append(ev[0].elapsed_time(ev[1]))
            st[["sample", "recount", "apply", "recount_alt", "mh_tables"][stage]] = float(np.median(ts))
        out[name]["stages_ms"] = st
    print(json.dumps(out), flush=True)
    # chunk-length sweep (the sampler's serial critical path is L steps per lane)
    for L in [int(x) for x in a.chunk_lens.split(",") if x]:
        del models
        torch.cuda.empty_cache()
        rl = common.build_and_train(dk, wk, None, vocab, a.topics, None, 0.01, 0x0D15EA5E, 0, L, None, train=False)
        m = GibbsLDA(rl.corpus, GibbsConfig(K=a.topics, count_mode="auto", sampler="lds" if a.lds else "auto"))
        m.initialize()
        m.sweep(a.burn)
        ts = []
        for _ in range(a.rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.sweep(a.sweeps)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / a.sweeps * 1e3)
        models = {}
        print(json.dumps({"chunk_len": L, "median_ms": float(np.median(ts)), "min_ms": float(np.min(ts)),
                          "slices": rl.corpus.n_slices, "long_docs": int(rl.corpus.long_rows.numel()),
                          "loglik": m.log_likelihood()}), flush=True)
        del m, rl
    return 0


if __name__ == "__main__":
    sys.exit(main())
