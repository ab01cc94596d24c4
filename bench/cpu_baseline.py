#!/usr/bin/env python3
"""Reference-equivalent CPU baseline for BASELINE.md (no GPU).

The reference's LDA stage is oni-lda-c ``lda est`` (variational EM, MPI over documents;
SURVEY.md §2.2 C22, §3.2) followed by a Spark post-LDA scoring pass (C24). This measures our
file-format-compatible C++ port-by-behaviour of that engine (csrc/lda_cpu, OpenMP over
documents = the MPI ranks' work on one host) on the SAME synthetic day bench.py uses, plus a
host (NumPy) θ·φ scoring pass, and prints one JSON line:

  records_per_sec_per_em_iter = flows × EM iterations / s   (the bench.py "value" analogue)
  score_records_per_sec       = flows / s of the host scoring pass

  python bench/cpu_baseline.py --flows 1000000 --em-iters 3 --threads 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--em-iters", type=int, default=3)
    ap.add_argument("--var-max-iter", type=int, default=20)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--em-convergence", type=float, default=0.0,
                    help="lda-c 'em convergence' (1e-4 = the lda-c settings default; 0 runs --em-iters)")
    ap.add_argument("--day", action="store_true",
                    help="time the whole day like bench.py's step: featurize -> corpus -> lda est -> score -> "
                         "top-3000 -> CSV rows (lda-c defaults: --em-iters 100 --em-convergence 1e-4)")
    a = ap.parse_args()
    if a.day and a.em_iters == 3:
        a.em_iters, a.em_convergence = 100, 1e-4
    import torch

    from oni355.models import vem
    from oni355.models.corpus import build_corpus
    from oni355.pipeline import common, flow
    from oni355.synth.flow import generate_flows

    torch.set_num_threads(a.threads)
    day = generate_flows(a.flows, seed=7, n_hosts=max(64, a.flows // 25))
    t_day = time.perf_counter()
    d = flow.to_device(day.cols, "cpu")
    cuts = flow.compute_cuts(d, None)
    sw, dw = flow.wordify(d, cuts)
    dk = torch.cat([common.u32_to_i64(d["sip"]), common.u32_to_i64(d["dip"])])
    wk = torch.cat([common.u32_to_i64(sw), common.u32_to_i64(dw)])
    vocab = common.global_vocab(wk, None)
    wid = torch.searchsorted(vocab, wk)
    udoc, inv = torch.unique(dk, return_inverse=True)
    c = build_corpus(inv, wid, int(udoc.numel()), int(vocab.numel()), common.i64_to_u32bits(udoc), 1, 128)
    doc_ptr = c.doc_pair_ptr.numpy().astype(np.int64)
    t_pre = time.perf_counter() - t_day
    t0 = time.perf_counter()
    res = vem.estimate(doc_ptr, c.pair_word.numpy(), c.pair_cnt.numpy(), c.V, a.topics, alpha=2.5,
                       estimate_alpha=True, var_max_iter=a.var_max_iter, var_convergence=1e-6,
                       em_max_iter=a.em_iters, em_convergence=a.em_convergence, threads=a.threads)
    dt = time.perf_counter() - t0
    iters = max(res.iterations, 1)
    # host scoring pass (the Spark post-LDA analogue): θ = normalised γ, φ = exp(log β)ᵀ
    theta = (res.gamma / res.gamma.sum(1, keepdims=True)).astype(np.float32)
    phi = np.exp(res.log_beta).T.astype(np.float32).copy()
    sdoc = torch.searchsorted(udoc, common.u32_to_i64(d["sip"])).numpy()
    ddoc = torch.searchsorted(udoc, common.u32_to_i64(d["dip"])).numpy()
    swid = torch.searchsorted(vocab, common.u32_to_i64(sw)).numpy()
    dwid = torch.searchsorted(vocab, common.u32_to_i64(dw)).numpy()
    t1 = time.perf_counter()
    s1 = np.einsum("ij,ij->i", theta[sdoc], phi[swid])
    s2 = np.einsum("ij,ij->i", theta[ddoc], phi[dwid])
    sc = np.minimum(s1, s2)
    keep = np.nonzero(sc < 1.0)[0]
    top = keep[np.argsort(sc[keep], kind="stable")[:3000]]
    st = time.perf_counter() - t1
    t2 = time.perf_counter()
    from oni355.io import results as rio
    rendered = rio.format_flow(day.cols, top, sw.numpy()[top].view(np.uint32), dw.numpy()[top].view(np.uint32),
                               s1[top], s2[top], sc[top])
    t_csv = time.perf_counter() - t2
    day_s = time.perf_counter() - t_day
    out = {"what": "reference-equivalent CPU path: C++ variational-EM lda est + host scoring",
           "flows": a.flows, "topics": a.topics, "threads": a.threads, "D": c.D, "V": c.V, "T": c.T,
           "nnz": c.nnz, "em_iters": iters, "em_s": round(dt, 3), "em_iters_per_sec": round(iters / dt, 4),
           "records_per_sec_per_em_iter": round(a.flows * iters / dt, 1),
           "score_s": round(st, 3), "score_records_per_sec": round(a.flows / st, 1), "top_n": int(top.size),
           "em_convergence": a.em_convergence, "var_max_iter": a.var_max_iter,
           "likelihood_last": [float(x) for x in np.asarray(res.likelihood).reshape(-1)[-3:]],
           "featurize_corpus_s": round(t_pre, 3), "csv_rows_s": round(t_csv, 3), "csv_rows": len(rendered),
           "day_s": round(day_s, 3), "flows_per_sec_day": round(a.flows / day_s, 1)}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
