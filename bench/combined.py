#!/usr/bin/env python3
"""Config 5 of BASELINE.json: combined flow + DNS + proxy day, one LDA model per source
(as ml_ops.sh runs one model per data source), K = 100 by default, data parallel over the node.

``--mode day`` (default): one timed *step* = the whole day of every source, as oni-ml runs it:
host columns → H2D → featurize → corpus → ``--sweeps`` Gibbs sweeps → score → top-N → CSV rows,
source after source; ``value`` = events of the node-wide day × steps / s (records fully scored per
second). ``--mode sweep``: one step = one Gibbs sweep of each of the three models (all three
resident in HBM, taking turns in chunks of ``--chunk`` sweeps); ``value`` = events × sweeps / s,
reported as record-sweeps/s. Both report per-model times, the measured HBM peak next to the sizing
model (oni355.utils.sizing) and its projection for the named 1B-event / 8-GPU configuration.

  python bench/combined.py                                   # 1 GPU, 12.5M flows + 6.25M DNS + 6.25M proxy
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/combined.py \
      --flows-per-gpu 62500000 --dns-per-gpu 31250000 --proxy-per-gpu 31250000   # the 1B-event day
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows-per-gpu", type=int, default=12_500_000)
    ap.add_argument("--dns-per-gpu", type=int, default=6_250_000)
    ap.add_argument("--proxy-per-gpu", type=int, default=6_250_000)
    ap.add_argument("--topics", type=int, default=100)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--chunk", type=int, default=10, help="sweeps per model between model switches")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--mode", choices=["day", "sweep"], default="day")
    ap.add_argument("--sweeps", type=int, default=200, help="day mode: Gibbs sweeps per model per day")
    ap.add_argument("--maxresults", type=int, default=3000)
    ap.add_argument("--flow-shards", type=int, default=1,
                    help="day mode: build the flow day from this many weak-scaling shards generated in parallel "
                         "processes (a 500M-flow / 1B-token flow model on one GPU)")
    ap.add_argument("--gen-procs", type=int, default=8, help="worker processes of --flow-shards generation")
    ap.add_argument("--recall-at", default="",
                    help="day mode: also report planted recall in the top N for these N (comma-separated, each "
                         "≤ --maxresults; e.g. the 1B-token day plants 200 anomalies per 62.5M-flow shard)")
    ap.add_argument("--realistic-vocab", action="store_true",
                    help="day mode: long-tail vocabularies on every source (flow V ~ 1.7e5 per 12.5M flows; dns / "
                         "proxy: half the rows from the long tail), as bench.py --realistic-vocab")
    a = ap.parse_args(argv)
    # --recall-at "3000,15000" (or "+"-separated: tools/gpu.sh splits at commas); the day then
    # selects max(N) result rows so the deeper recalls can be read off the same ranking
    a.recall_ns = [int(x) for x in a.recall_at.replace("+", ",").split(",") if x] if a.recall_at else []
    if a.mode == "day" and a.steps == 20 and a.warmup == 10:
        a.steps, a.warmup = 2, 1
    # the contract is ONE JSON line on stdout: keep the real stdout for it and send everything else
    # written to fd 1 (RCCL's version banner at communicator creation, library chatter) to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch

    from oni355.utils.obs import heartbeat_from_env, stack_dumps_from_env
    stack_dumps_from_env()
    heartbeat_from_env()

    from oni355.parallel import comm as pc
    from oni355.pipeline.synthetic import build_source
    from oni355.utils import sizing

    comm = pc.init_from_env(a.device)
    dev = comm.device
    cuda = dev.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    if a.mode == "day":
        out = run_day_mode(a, comm, sync)
        if comm.rank == 0:
            print(json.dumps(out), file=json_out, flush=True)
        pc.shutdown()
        return 0

    t0 = time.perf_counter()
    sources = []
    for src, per in (("flow", a.flows_per_gpu), ("dns", a.dns_per_gpu), ("proxy", a.proxy_per_gpu)):
        if per <= 0:
            continue
        su = build_source(src, per, a.topics, comm, seed=a.seed)
        sync()
        su.model.initialize()
        sync()
        sources.append(su)
        su.day = None  # host columns are no longer needed
        print(f"[combined] {src}: {per} events/rank ready at {time.perf_counter() - t0:.1f} s", file=sys.stderr,
              flush=True)
    sync()
    setup_s = time.perf_counter() - t0
    for su in sources:
        su.model.sweep(a.warmup)
    sync()
    comm.barrier()
    per_model = {}
    t0 = time.perf_counter()
    # each model runs its sweeps in chunks (graph-replayed pairs, one health check per chunk),
    # as oni-ml runs a model's sweeps back to back; the total work is a.steps sweeps per model
    done = 0
    while done < a.steps:
        n = min(a.chunk, a.steps - done)
        for su in sources:
            su.model.sweep(n)
        done += n
    sync()
    comm.barrier()
    dt = comm.allreduce_scalar(time.perf_counter() - t0, "max")
    # per-model sweep time, measured separately after the combined loop
    for su in sources:
        sync()
        t1 = time.perf_counter()
        su.model.sweep(4)
        sync()
        per_model[su.source] = round(comm.allreduce_scalar(time.perf_counter() - t1, "max") / 4 * 1e3, 4)
    events = sum(su.n_total for su in sources)
    plans = [sizing.plan(su.source, su.per_rank, su.K, su.run.corpus.D, int(su.vocab.numel()),
                         0 if su.source == "flow" else 48) for su in sources]
    peak = torch.cuda.max_memory_allocated(dev) if cuda else 0
    projection = sizing.plan_combined(1_000_000_000, 8, a.topics)
    out = {
        "metric": f"combined flow+dns+proxy record-sweeps/sec (whole node), {a.topics}-topic LDA x3",
        "value": round(events * a.steps / dt, 1), "unit": "records*sweeps/s", "n_gpus": comm.world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "dtype": "fp32", "data": "synthetic flow/dns/proxy (oni355.synth)",
        "config": {"model": "oni-suspicious-connects-combined-lda", "topics": a.topics, "global_batch": events,
                   "events_per_gpu": {su.source: su.per_rank for su in sources},
                   "parallelism": f"dp{comm.world}",
                   "baseline_config": "Combined flow+DNS+proxy 1B events, 100 topics, 8xMI355X (weak-scaled)"},
        "ms_per_sweep_by_model": per_model,
        "tokens": {su.source: int(comm.allreduce_scalar(su.run.corpus.T, "sum")) for su in sources},
        "vocab": {su.source: int(su.vocab.numel()) for su in sources},
        "hbm_peak_GB_measured": round(peak / 1e9, 3),
        "hbm_plan_GB": [p.as_dict() for p in plans],
        "projection_1B_events_8gpu": {"per_gpu_peak_GB": round(sum(p.steady_bytes for p in projection) / 1e9
                                                               + max(p.peak_bytes - p.steady_bytes
                                                                     for p in projection) / 1e9, 2),
                                      "fits_288GB": all(p.fits() for p in projection)},
        "setup_s": round(setup_s, 2),
    }
    if comm.rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    pc.shutdown()
    return 0


def run_day_mode(a, comm, sync) -> dict:
    """Every source's whole day per step (see the module docstring)."""
    import tempfile

    import torch

    from oni355 import schema
    from oni355.io import results as rio
    from oni355.utils import sizing

    dev = comm.device
    rank, world = comm.rank, comm.world
    t0 = time.perf_counter()
    days = []
    for src, per in (("flow", a.flows_per_gpu), ("dns", a.dns_per_gpu), ("proxy", a.proxy_per_gpu)):
        if per <= 0:
            continue
        n_total = per * world
        wide = 0.5 if a.realistic_vocab else 0.0
        if src == "flow" and a.flow_shards > 1:
            from oni355.synth.flow import generate_flows_sharded
            if world > 1 or per % a.flow_shards:
                raise SystemExit("--flow-shards: one rank, flows divisible by the shard count")
            day = generate_flows_sharded(per // a.flow_shards, a.flow_shards, seed=a.seed, n_hosts=max(64, n_total // 25),
                                         procs=a.gen_procs, wide_vocab=a.realistic_vocab)
        elif src == "flow":
            from oni355.synth.flow import generate_flows
            day = generate_flows(per, seed=a.seed, rank=rank, n_hosts=max(64, n_total // 25),
                                 wide_vocab=a.realistic_vocab)
        elif src == "dns":
            from oni355.synth.dns import generate_dns
            day = generate_dns(per, seed=a.seed, rank=rank, n_clients=max(32, n_total // 40), wide_vocab=wide)
        else:
            from oni355.synth.proxy import generate_proxy
            day = generate_proxy(per, seed=a.seed, rank=rank, n_clients=max(32, n_total // 40), wide_vocab=wide)
        days.append((src, per, n_total, day))
        print(f"[combined] {src}: {per} events/rank generated at {time.perf_counter() - t0:.1f} s", file=sys.stderr,
              flush=True)
    setup_s = time.perf_counter() - t0
    tmp = tempfile.mkdtemp(prefix="oni_combined_")

    def one_day():
        times, stats = {}, {}
        for src, per, n_total, day in days:
            kw = dict(K=a.topics, sweeps=a.sweeps, tol=1.0, maxresults=max([a.maxresults] + a.recall_ns), device=dev, comm=comm,
                      row_offset=rank * per)
            ts = time.perf_counter()
            if src == "flow":
                from oni355.pipeline.flow import run_flow
                res = run_flow(day.cols, **kw)
            elif src == "dns":
                from oni355.pipeline.dns import run_dns
                res = run_dns(day.cols, top_domains=day.top_domains, user_domain="intel", **kw)
            else:
                from oni355.pipeline.proxy import run_proxy
                res = run_proxy(day.cols, **kw)
            rendered = rio.render_result(src, day.cols, res, rank * per, comm)
            if rank == 0:
                rio.write_rendered(os.path.join(tmp, f"{src}_results.csv"), schema.result_columns(src), rendered)
            sync()
            times[src] = time.perf_counter() - ts
            m = res.lda.model
            stats[src] = {"train_dev_s": res.timings.get("train_dev_s", res.timings.get("train_s")),
                          "tokens": res.lda.corpus.T, "vocab": int(res.lda.vocab.numel()),
                          "sampler": m.chain["sampler"], "mh_burn": m.chain["mh_burn"],
                          "max_topic_share": round(float(m.nk_cur[: m.K].max()) / max(m.T_global, 1), 4),
                          "max_word_tokens": int(m.nwk[:, : m.K].sum(1, dtype=torch.int64).max()),
                          "posterior_sum_dtypes": ({k: str(m._avg[k].dtype) for k in ("wk", "k", "dk")}
                                                   if m._avg is not None and m._avg["wk"] is not None else None),
                          "min_score_topN": float(res.scores[0]) if len(res.scores) else None,
                          "n_scores_nonpositive": int((np.asarray(res.scores) <= 0).sum()),
                          "rows": len(rendered), "loglik": res.stats.get("loglik"),
                          "planted_recall_topN": float(np.isin(day.anomaly_rows + rank * per,
                                                               res.rows[: a.maxresults]).mean())}
            if a.recall_at:
                pl = day.anomaly_rows + rank * per
                stats[src]["planted_recall_at"] = {str(n): round(float(np.isin(pl, res.rows[:n]).mean()), 4)
                                                   for n in a.recall_ns}
                stats[src]["planted"] = int(pl.size)
            del res
            print(f"[combined] {src} day {times[src]:.3f} s", file=sys.stderr, flush=True)
        return times, stats

    import numpy as np
    for _ in range(a.warmup):
        one_day()
    sync()
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.reset_peak_memory_stats(dev)
    per_step = []
    t1 = time.perf_counter()
    for _ in range(a.steps):
        per_step.append(one_day())
    sync()
    comm.barrier()
    dt = comm.allreduce_scalar(time.perf_counter() - t1, "max")
    events = sum(n_total for _, _, n_total, _ in days)
    peak = torch.cuda.max_memory_allocated(dev) if dev.type == "cuda" else 0
    times, stats = per_step[-1]
    projection = sizing.plan_combined(1_000_000_000, 8, a.topics)
    return {
        "metric": f"combined flow+dns+proxy records scored/sec (whole node), {a.topics}-topic LDA x3",
        "value": round(events * a.steps / dt, 1), "unit": "records/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "dtype": "fp32", "data": "synthetic flow/dns/proxy (oni355.synth)",
        "config": {"model": "oni-suspicious-connects-combined-lda", "topics": a.topics, "global_batch": events,
                   "events_per_gpu": {src: per for src, per, _, _ in days}, "parallelism": f"dp{world}",
                   "sweeps_per_model": a.sweeps, "maxresults": a.maxresults,
                   "baseline_config": "Combined flow+DNS+proxy 1B events, 100 topics, 8xMI355X (one GPU's share)"},
        "realistic_vocab": a.realistic_vocab,
        "step": f"each source's whole day (H2D -> featurize -> corpus -> {a.sweeps} sweeps -> score -> "
                f"top-{a.maxresults} -> CSV rows), source after source",
        "day_s_by_model": {k: round(v, 4) for k, v in times.items()},
        "ms_per_sweep_in_training_by_model": {k: round(v["train_dev_s"] / a.sweeps * 1e3, 4)
                                              for k, v in stats.items() if v["train_dev_s"]},
        "model_stats": stats,
        "hbm_peak_GB_measured": round(peak / 1e9, 3),
        "projection_1B_events_8gpu": {"per_gpu_peak_GB": round(sum(p.steady_bytes for p in projection) / 1e9
                                                               + max(p.peak_bytes - p.steady_bytes
                                                                     for p in projection) / 1e9, 2),
                                      "fits_288GB": all(p.fits() for p in projection)},
        "setup_s": round(setup_s, 2),
    }


if __name__ == "__main__":
    sys.exit(main())
