#!/usr/bin/env python3
"""Headline benchmark: netflow suspicious-connects, 20-topic collapsed-Gibbs LDA on MI355X.

Metric (BASELINE.json): "netflow records scored/sec (whole node) + Gibbs iters/sec, 20-topic LDA".
One timed *step* = one full Gibbs sweep over every token of the day (2 tokens per flow) including
the per-sweep RCCL all-reduce of Δn_wk and the q-table refresh. ``value`` = whole-node netflow
records swept per second (= total flows × sweeps/s). Also reported: Gibbs iters/s, tokens/s and
the post-LDA scoring pass (records scored/s: θ·φ score of every flow + top-N selection).

Weak scaling: every GPU owns ``--flows-per-gpu`` synthetic flows (default 12.5M, so N=8 is the
BASELINE config "Netflow 100M flows, 20 topics, DP=8"). Synthetic data with random-init topic
priors (oni355.synth.flow), random-init LDA. Launch for N>1:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# Reference-equivalent CPU path (C++ variational-EM lda est on this host's 8 cores, same synthetic
# 12.5M-flow day): flows × EM iterations / s. BASELINE.md "Measured baselines";
# profiles/r1_cpu_baseline_12.5M.json; reproduce with bench/cpu_baseline.py.
BASELINE_RECORDS_PER_SEC = 889_887.5


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--flows-per-gpu", type=int, default=12_500_000)
    ap.add_argument("--topics", type=int, default=None)
    ap.add_argument("--source", choices=["flow", "dns", "proxy"], default="flow")
    ap.add_argument("--score-path", choices=["tiles", "pairs", "pairs_unsorted", "gather"], default="pairs",
                    help="tiles: distinct pairs as 16x16 MFMA blocks; pairs: per-pair VALU dots; "
                         "gather: per-event θ/φ row gathers (tiles/pairs + 4-B per-event pair gathers)")
    ap.add_argument("--events-per-gpu", type=int, default=2_000_000, help="dns/proxy events per GPU")
    ap.add_argument("--chunk-len", type=int, default=0, help="0 = auto (global token count)")
    ap.add_argument("--maxresults", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args(argv)
    a.topics_set = a.topics is not None
    if a.topics is None:
        a.topics = 20

    # the contract is ONE JSON line on stdout: keep the real stdout for it and send everything else
    # written to fd 1 (RCCL's version banner at communicator creation, library chatter) to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch

    from oni355.utils.obs import stack_dumps_from_env
    stack_dumps_from_env()

    from oni355.parallel import comm as pc
    from oni355.pipeline import common

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        if a.gpus > 1:
            print(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}; launch with torch.distributed.run", file=sys.stderr)
            return 2
    if a.no_graph:
        os.environ["ONI_NO_GRAPH"] = "1"
    comm = pc.init_from_env(a.device)
    dev = comm.device
    rank, world = comm.rank, comm.world

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    t_setup = time.perf_counter()
    from oni355 import ops
    from oni355.pipeline.synthetic import build_source
    # flows: hosts scale with the node-wide day so N=8 is one 100M-flow day split over 8 ranks
    per = a.flows_per_gpu if a.source == "flow" else a.events_per_gpu
    K = a.topics if (a.source == "flow" or a.topics_set) else 50
    su = build_source(a.source, per, K, comm, seed=a.seed, chunk_len=a.chunk_len)
    n_total, day, sides, vocab, run = su.n_total, su.day, su.sides, su.vocab, su.run
    model = run.model
    model.initialize()
    sync()
    setup_s = time.perf_counter() - t_setup

    # ---- warmup + timed sweeps -----------------------------------------------------------------
    model.sweep(a.warmup)
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    model.sweep(a.steps)
    sync()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt = comm.allreduce_scalar(dt, "max")

    # ---- post-LDA scoring pass (records scored/s), timed separately --------------------------
    dkeys, theta = common.gather_theta(run, comm)
    phi = model.phi()
    # distinct (doc, word) pairs + per-endpoint pair index: built once per day (corpus dictionaries)
    plans = {"tiles": common.score_plan(dkeys, vocab, sides, tiles=True),
             "pairs": common.score_plan(dkeys, vocab, sides, tiles=False),
             "pairs_unsorted": common.score_plan(dkeys, vocab, sides, tiles=False, sort_events=False)}
    lk = [(common.lookup(dkeys, dk_), common.lookup(vocab, wk_)) for dk_, wk_ in sides]

    def score_once(path):
        hist = torch.zeros(2048, dtype=torch.int32, device=dev)
        if path in plans:
            sc, _, _ = common.plan_score(theta, phi, plans[path], 1.0, hist=hist)
        elif len(lk) == 2:
            sc, _, _ = ops.score(theta, phi, lk[0][0], lk[0][1], lk[1][0], lk[1][1], tol=1.0, hist=hist)
        else:
            sc, _, _ = ops.score(theta, phi, lk[0][0], lk[0][1], tol=1.0, hist=hist)
        order = plans[path].order if path in plans else None
        return common.top_n(sc, 1.0, a.maxresults, comm, rank * per, hist=hist, order=order)

    def time_path(path, reps=5):
        score_once(path)
        sync()
        comm.barrier()
        t1 = time.perf_counter()
        for _ in range(reps):
            res = score_once(path)
        sync()
        comm.barrier()
        return comm.allreduce_scalar((time.perf_counter() - t1) / reps, "max"), res

    score_ab = {p: round(time_path(p)[0] * 1e3, 3) for p in ("tiles", "pairs", "pairs_unsorted", "gather")
                if p != a.score_path}
    score_dt, (rows, scs) = time_path(a.score_path)
    plan = plans["tiles"]
    ll = model.log_likelihood()

    tokens_local = run.corpus.T
    tokens = int(comm.allreduce_scalar(tokens_local, "sum"))
    ms = dt / a.steps * 1e3
    value = n_total * a.steps / dt
    planted = day.anomaly_rows + rank * per
    hits = np.isin(planted, rows.cpu().numpy()[: a.maxresults])
    hit_frac = comm.allreduce_scalar(float(hits.sum()), "sum") / max(comm.allreduce_scalar(float(planted.size), "sum"), 1)
    metric = "netflow records scored/sec (whole node) + Gibbs iters/sec, 20-topic LDA"
    if a.source != "flow":
        metric = f"{a.source} records scored/sec (whole node) + Gibbs iters/sec, {K}-topic LDA"
    out = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "records/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / BASELINE_RECORDS_PER_SEC, 1) if a.source == "flow" else None,
        "dtype": "fp32",
        "data": f"synthetic {a.source} (oni355.synth.{a.source}: random-init topic priors, Zipf hosts, planted anomalies)",
        "config": {"model": f"oni-suspicious-connects-{a.source}-lda", "topics": K, "global_batch": n_total,
                   "events_per_gpu": per, "seq_len": 2 if a.source == "flow" else 1, "parallelism": f"dp{world}",
                   "baseline_config": ("Netflow 100M flows, 20 topics, DP=8 (N=8); weak-scaled 12.5M flows/GPU"
                                       if a.source == "flow" else
                                       "DNS suspicious-connects (pcap->word pipeline), 50 topics"
                                       if a.source == "dns" else "proxy suspicious-connects")},
        "gibbs_iters_per_sec": round(a.steps / dt, 3),
        "tokens_per_sec": round(tokens * a.steps / dt, 1),
        "tokens": tokens,
        "vocab": int(vocab.numel()),
        "docs_local": run.corpus.D,
        "score_records_per_sec": round(n_total / score_dt, 1),
        "score_ms": round(score_dt * 1e3, 3),
        "score_path": a.score_path,
        "score_ms_other_paths": score_ab,
        "score_pairs": plan.n_pairs,
        "score_mfma_items": plan.tiles.n_items,
        "score_mfma_block_density": round(plan.tiles.density(), 4),
        "loglik": ll,
        "planted_anomaly_recall_topN": round(hit_frac, 4),
        "setup_s": round(setup_s, 2),
        "allreduce_s_per_sweep": (model.timings["allreduce_s"] / max(model.timings["allreduce_calls"], 1)),
    }
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    pc.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
