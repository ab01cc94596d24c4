#!/usr/bin/env python3
"""Headline benchmark: netflow suspicious-connects with 20-topic collapsed-Gibbs LDA on MI355X.

Metric (BASELINE.json): "netflow records scored/sec (whole node) + Gibbs iters/sec, 20-topic LDA".

One timed *step* (default ``--mode pipeline``) is one complete ``oni-ml YYYYMMDD flow`` day run on
every rank's shard — exactly what the CLI executes (oni355.pipeline.flow.run_flow), from the
day's raw columns in host memory to the rendered, globally ordered top-N result rows (CSV written
by rank 0):

    H2D → quantile cuts (K01, X03) → flow words (K03) → vocabulary (K08, X02) → owner routing →
    corpus CSR + SELL (K09) → LDA init + ``--sweeps`` Gibbs sweeps (K10-K12, X01 per sweep) →
    θ/φ (K13, X05) → score plan + scores (K15) → top-N (K16, X06) → CSV rows.

``value`` = whole-node flows fully processed (scored) per second = global flows × steps / time.
``gibbs_iters_per_sec`` = sweeps of the in-step training / its device time (median over steps).
``--mode sweep`` times bare sweeps of an already built model instead (the round-1 measurement,
reported as flow-sweeps/s under a different metric name; for sampler A/B work).

Weak scaling: every GPU owns ``--flows-per-gpu`` synthetic flows (default 12.5M, so N=8 is the
BASELINE config "Netflow 100M flows, 20 topics, DP=8"). Synthetic data with random-init topic
priors (oni355.synth.flow), random-init LDA. ``--gpus N`` outside torchrun re-launches itself
under ``torch.distributed.run`` (a child process, started before anything touches the GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "netflow records scored/sec (whole node) + Gibbs iters/sec, 20-topic LDA"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=["pipeline", "sweep"], default="pipeline")
    ap.add_argument("--sweeps", type=int, default=200, help="Gibbs sweeps per pipeline step (oni-ml default)")
    ap.add_argument("--flows-per-gpu", type=int, default=12_500_000)
    ap.add_argument("--events-per-gpu", type=int, default=2_000_000, help="dns/proxy events per GPU")
    ap.add_argument("--topics", type=int, default=None)
    ap.add_argument("--source", choices=["flow", "dns", "proxy"], default="flow")
    ap.add_argument("--from-pcap", action="store_true",
                    help="dns: every step decodes the shard's pcap file (config 3 'pcap→word pipeline')")
    ap.add_argument("--realistic-vocab", action="store_true",
                    help="long-tail synthetic vocabulary (SURVEY §7.5 sizing): flow -- service ports and wider "
                         "bins (V ~ 4e5); dns / proxy -- half the rows from the long tail of record types, "
                         "rcodes, name shapes / methods, content types, statuses, user agents, URIs")
    ap.add_argument("--lt-codebook", type=float, default=0.01,
                    help="flow --realistic-vocab: long-tail behaviours per flow (0.01 -> V ~ 1.7e5 at 12.5M "
                         "flows, 0.04 -> V ~ 4-5e5)")
    ap.add_argument("--chunk-len", type=int, default=0, help="0 = auto (global token count)")
    ap.add_argument("--maxresults", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--beta", type=float, default=None, help="LDA β (default: the pipeline's)")
    ap.add_argument("--env", action="append", default=[], metavar="KEY=VALUE",
                    help="set an ONI_* environment knob for this run (A/B runs; repeatable)")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--prefetch-at", choices=["start", "train"], default="start",
                    help="when the next day's upload is queued: at step start (default) or as the sweeps "
                         "start (measured 8 ms slower: the sweeps run slower beside the upload)")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="upload (and, --from-pcap, decode) each day inside its step instead of overlapping "
                         "it with the previous day's compute")
    ap.add_argument("--from-store", action="store_true",
                    help="every step reads its day from the columnar store (memory-mapped read + IPv6 keying + "
                         "pinned copy on a loader thread, overlapping the previous day) -- what oni-ml does day "
                         "after day (pipeline.daily); the store is written once at setup")
    ap.add_argument("--realistic-steps", type=int, default=3,
                    help="after the headline, also time this many steps (1 warm-up) of the realistic-vocabulary "
                         "day of the same size and report them under 'realistic_vocab' (0: skip)")
    a = ap.parse_args(argv)
    for kv in a.env:
        k, _, v = kv.partition("=")
        if not k.startswith("ONI_"):
            raise SystemExit(f"--env takes ONI_* knobs, not {k}")
        os.environ[k] = v
    a.topics_set = a.topics is not None
    if a.topics is None:
        a.topics = 20 if a.source != "dns" else 50
    return a


def relaunch(n: int, argv: list[str]) -> int:
    """Start N ranks under torch.distributed.run as a CHILD process (never an exec)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch(a.gpus, argv)

    # the contract is ONE JSON line on stdout: keep the real stdout for it and send everything else
    # written to fd 1 (RCCL's version banner at communicator creation, library chatter) to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch

    from oni355.utils.obs import stack_dumps_from_env, heartbeat_from_env
    stack_dumps_from_env()
    heartbeat_from_env()

    from oni355.parallel import comm as pc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if a.no_graph:
        os.environ["ONI_NO_GRAPH"] = "1"
    comm = pc.init_from_env(a.device)
    out = run_sweep_mode(a, comm) if a.mode == "sweep" else run_pipeline_mode(a, comm)
    if (a.mode == "pipeline" and a.realistic_steps > 0 and not a.realistic_vocab and not a.from_pcap
            and not a.from_store):
        # the same day shape with a long-tail vocabulary (V ~ 4e5 flow words: the q table leaves
        # L2), reported next to the headline, not instead of it
        import copy
        b = copy.copy(a)
        b.realistic_vocab, b.steps, b.warmup = True, a.realistic_steps, 1
        r = run_pipeline_mode(b, comm)
        out["realistic_vocab"] = {k: r[k] for k in ("value", "ms_per_step", "ms_per_sweep_in_training", "vocab",
                                                    "tokens", "planted_anomaly_recall_topN", "steps", "warmup",
                                                    "stage_median_s")}
    if comm.rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    pc.shutdown()
    return 0


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _median_timings(per_step: list[dict]) -> dict:
    keys = [k for k in per_step[0] if k.endswith("_s")]
    return {k: round(statistics.median(t[k] for t in per_step), 5) for k in keys}


# -------------------------------------------------------------------------------------------------
def make_shard(a, comm):
    """This rank's shard of the synthetic day (host columns) + its global row offset."""
    rank, world = comm.rank, comm.world
    per = a.flows_per_gpu if a.source == "flow" else a.events_per_gpu
    n_total = per * world
    if a.source == "flow":
        from oni355.synth.flow import generate_flows
        day = generate_flows(per, seed=a.seed, rank=rank, n_hosts=max(64, n_total // 25),
                             wide_vocab=a.realistic_vocab, lt_codebook=a.lt_codebook)
    elif a.source == "dns":
        from oni355.synth.dns import generate_dns
        day = generate_dns(per, seed=a.seed, rank=rank, n_clients=max(32, n_total // 40),
                           wide_vocab=0.5 if a.realistic_vocab else 0.0)
    else:
        from oni355.synth.proxy import generate_proxy
        day = generate_proxy(per, seed=a.seed, rank=rank, n_clients=max(32, n_total // 40),
                             wide_vocab=0.5 if a.realistic_vocab else 0.0)
    return day, per, n_total


def run_pipeline_mode(a, comm) -> dict:
    import torch

    from oni355 import schema
    from oni355.io import results as rio

    dev = comm.device
    rank, world = comm.rank, comm.world
    t_setup = time.perf_counter()
    day, per, n_total = make_shard(a, comm)
    row_off = rank * per
    tmp = tempfile.mkdtemp(prefix="oni_bench_")
    pcap = None
    if a.source == "dns" and a.from_pcap:
        from oni355.synth.dns import write_pcap
        pcap = os.path.join(tmp, f"dns_rank{rank}.pcap")
        write_pcap(day, pcap)
    top = day.top_domains if a.source == "dns" else None

    kw = dict(K=a.topics, sweeps=a.sweeps, tol=1.0, maxresults=a.maxresults, chunk_len=a.chunk_len, device=dev,
              comm=comm, row_offset=row_off)
    if a.beta is not None:
        kw["beta"] = a.beta
    # flow days stream in through a double-buffered prefetcher: the loader's pinned buffers are
    # uploaded on a copy stream while the previous day computes (every step still uploads its day)
    pf, pinned, ahead = None, None, None
    if pcap is not None:
        from oni355.io.decoders import read_pcap_dns
        if not a.no_prefetch:
            # every step decodes its day's pcap; the decode of day k+1 runs on a host thread while
            # day k computes
            from oni355.io.staging import HostAhead
            ahead = HostAhead(read_pcap_dns, pcap)
    store_pipe = None
    if a.from_store:
        # the product path: oni-ml's day pipeline over a stored day (re-read every step)
        from oni355.io.staging import PinnedSlots
        from oni355.pipeline.daily import DayPipeline, load_host_day
        from oni355.store import columnar
        root = os.path.join(tmp, "store")
        columnar.write_day(root, a.source, "20160708", {k: v for k, v in day.cols.items() if not k.startswith("_")})
        slots = PinnedSlots() if dev.type == "cuda" else None

        def _load(date):
            h = load_host_day(a.source, root, date, 0, 1, dev, None, None, slots=slots)
            h.row_off = row_off
            return h
        store_pipe = DayPipeline(_load, dev, slots)
        store_pipe.extend(["20160708"] * (a.warmup + a.steps))
    if dev.type == "cuda" and not a.no_prefetch and pcap is None and store_pipe is None:
        from oni355.io.staging import Prefetcher
        if a.source == "flow":
            from oni355.pipeline.flow import DEVICE_COLS
            pinned = Prefetcher.pin(day.cols, DEVICE_COLS)
        elif a.source == "dns":
            from oni355.pipeline.dns import host_arrays
            pinned = Prefetcher.pin_arrays(host_arrays(day.cols))
        else:
            from oni355.pipeline.proxy import host_arrays
            pinned = Prefetcher.pin_arrays(host_arrays(day.cols))
        pf = Prefetcher(dev)
        pf.submit(pinned)
    setup_s = time.perf_counter() - t_setup

    def step():
        t0 = time.perf_counter()
        dcols, on_train = None, None
        if store_pipe is not None:
            from oni355.pipeline.daily import run_day
            w0 = store_pipe.wait_s
            hday, dcols = store_pipe.take()
            kw2 = dict(kw)
            kw2.pop("comm")
            kw2.pop("row_offset")
            if a.source == "dns":
                kw2.update(top_domains=top, user_domain="intel")
            res = run_day(a.source, hday, dcols, comm, kw2)
            res.timings["store_load_s"] = hday.load_s
            res.timings["loader_wait_s"] = store_pipe.wait_s - w0
            if store_pipe.pf is not None:
                res.timings["h2d_copy_dev_s"] = (store_pipe.pf.copy_ms() or 0.0) / 1e3
            t1 = time.perf_counter()
            results.submit(hday.cols, res, row_off)
            res.timings["results_s"] = time.perf_counter() - t1
            return res
        if pf is not None:
            dcols = pf.take()
            # the next day's upload overlaps this day's compute
            if a.prefetch_at == "start" or a.source != "flow":
                pf.submit(pinned)
            else:
                on_train = lambda: pf.submit(pinned)  # noqa: E731
        if a.source == "flow":
            from oni355.pipeline.flow import run_flow
            cols = day.cols
            res = run_flow(cols, device_cols=dcols, on_train=on_train, **kw)
        elif a.source == "dns":
            from oni355.pipeline.dns import run_dns
            if pcap is not None:
                cols = ahead.take() if ahead is not None else read_pcap_dns(pcap)
            else:
                cols = day.cols
            t_dec = time.perf_counter() - t0
            res = run_dns(cols, top_domains=top, user_domain="intel", device_cols=dcols, **kw)
            res.timings["decode_s"] = t_dec
        else:
            from oni355.pipeline.proxy import run_proxy
            cols = day.cols
            res = run_proxy(cols, device_cols=dcols, **kw)
        if pf is not None:
            res.timings["h2d_copy_dev_s"] = pf.copy_ms() / 1e3
        t1 = time.perf_counter()
        # this day's rows are formatted on a worker thread while the next day computes; the
        # previous day's gather + CSV write happen here (the last day's at the drain below)
        results.submit(cols, res, row_off)
        res.timings["results_s"] = time.perf_counter() - t1
        return res

    csv_path = os.path.join(tmp, f"{a.source}_results.csv")
    header = schema.result_columns(a.source)
    results = rio.ResultPipe(a.source, comm, write=(lambda r: rio.write_rendered(csv_path, header, r))
                             if rank == 0 else None)

    for _ in range(a.warmup):
        step()
    results.drain()
    _sync(dev)
    comm.barrier()
    _sync(dev)
    per_step, res = [], None
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ts = time.perf_counter()
        res = step()
        res.timings["step_s"] = time.perf_counter() - ts
        per_step.append(res.timings)
    results.drain()  # the last day's rows are part of the timed work
    _sync(dev)
    results.close()
    if store_pipe is not None:
        store_pipe.close()
    comm.barrier()
    _sync(dev)
    dt = comm.allreduce_scalar(time.perf_counter() - t0, "max")

    med = _median_timings(per_step)
    # device time of the in-step training on a GPU (HIP events), host wall time on the CPU path
    train_s = comm.allreduce_scalar(med.get("train_dev_s", med.get("train_s", 0.0)), "max")
    model = res.lda.model
    tokens = int(comm.allreduce_scalar(res.lda.corpus.T, "sum"))
    planted = day.anomaly_rows + row_off
    hits = np.isin(planted, res.rows[: a.maxresults])
    hit_frac = comm.allreduce_scalar(float(hits.sum()), "sum") / max(comm.allreduce_scalar(float(planted.size), "sum"), 1)
    value = n_total * a.steps / dt
    K = a.topics
    metric = (METRIC if a.source == "flow" and K == 20 else
              f"{'netflow' if a.source == 'flow' else a.source} records scored/sec (whole node) + Gibbs iters/sec, "
              f"{K}-topic LDA")
    baseline_cfg = {"flow": "Netflow 100M flows, 20 topics, DP=8 (N=8); weak-scaled 12.5M flows/GPU",
                    "dns": "DNS suspicious-connects (pcap->word pipeline), 50 topics",
                    "proxy": "proxy suspicious-connects"}[a.source]
    return {
        "metric": metric,
        "value": round(value, 1),
        "unit": "records/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        # the reference publishes no number; the CPU reference-equivalent
        # measurement lives in BASELINE.md and is not comparable work per iteration
        "vs_baseline": None,
        "dtype": "fp32",
        "data": f"synthetic {a.source} (oni355.synth.{a.source}: random-init topic priors, Zipf hosts, planted anomalies)"
                + (", decoded from pcap every step" if pcap else "")
                + (", realistic (long-tail) vocabulary" if a.realistic_vocab else "")
                + (", read from the columnar store every step" if a.from_store else ""),
        "config": {"model": f"oni-suspicious-connects-{a.source}-lda", "topics": K, "global_batch": n_total,
                   "events_per_gpu": per, "seq_len": 2 if a.source == "flow" else 1, "parallelism": f"dp{world}",
                   "sweeps_per_step": a.sweeps, "maxresults": a.maxresults, "baseline_config": baseline_cfg},
        "step": ("one full oni-ml day per step, read from the columnar store (memory-mapped read, pinned copy "
                 "and H2D of day k+1 on a loader thread / copy stream during day k) -> " if a.from_store else "")
                + "one full oni-ml day run per step: host columns -> H2D -> featurize -> corpus -> "
                f"{a.sweeps} Gibbs sweeps -> score -> top-{a.maxresults} -> CSV rows"
                + ("; each step's H2D upload runs on a copy stream during the previous step" if pf is not None else "")
                + ("; each step's pcap decode runs on a host thread during the previous step" if ahead is not None
                   else "")
                + "; each step's result rows are formatted on a host thread during the next step (the last "
                  "step's inside the timed region)",
        "gibbs_iters_per_sec": round(a.sweeps / train_s, 2) if train_s > 0 else None,
        "ms_per_sweep_in_training": round(train_s / a.sweeps * 1e3, 4) if train_s > 0 else None,
        "tokens_per_sec_training": round(tokens * a.sweeps / train_s, 1) if train_s > 0 else None,
        "stage_median_s": med,
        "tokens": tokens,
        "vocab": int(res.lda.vocab.numel()),
        "docs_local": res.lda.corpus.D,
        "loglik": model.likelihoods[-1][1] if model.likelihoods else None,
        "planted_anomaly_recall_topN": round(hit_frac, 4),
        "setup_s": round(setup_s, 2),
        "allreduce_ms_per_sweep": model.allreduce_ms_per_sweep(),
        "allreduce_bytes_per_sweep": model.allreduce_bytes_per_sweep(),
        # the auto count mode's measured changed-token fractions (sweep, fraction), last few
        "changed_fraction_tail": [(int(a_), round(float(b_), 4)) for a_, b_ in model.change_log[-3:]],
        # count magnitudes (the int32 tables' headroom) and the device memory high-water mark
        "max_topic_share": round(float(model.nk_cur[:K].max()) / max(model.T_global, 1), 4),
        "min_score_topN": float(res.scores[0]) if len(res.scores) else None,
        "hbm_peak_gb": (round(torch.cuda.max_memory_allocated(dev) / 2**30, 2) if dev.type == "cuda" else None),
    }


# -------------------------------------------------------------------------------------------------
def run_sweep_mode(a, comm) -> dict:
    """Bare sweeps of an already built model (round-1 measurement): flows × sweeps / s."""
    from oni355.pipeline.synthetic import build_source
    dev = comm.device
    world = comm.world
    t_setup = time.perf_counter()
    per = a.flows_per_gpu if a.source == "flow" else a.events_per_gpu
    su = build_source(a.source, per, a.topics, comm, seed=a.seed, chunk_len=a.chunk_len)
    model = su.run.model
    model.initialize()
    _sync(dev)
    setup_s = time.perf_counter() - t_setup
    model.sweep(a.warmup)
    _sync(dev)
    comm.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    model.sweep(a.steps)
    _sync(dev)
    comm.barrier()
    _sync(dev)
    dt = comm.allreduce_scalar(time.perf_counter() - t0, "max")
    tokens = int(comm.allreduce_scalar(su.run.corpus.T, "sum"))
    return {
        "metric": f"{a.source} record-sweeps/sec (whole node), {a.topics}-topic collapsed-Gibbs LDA",
        "value": round(su.n_total * a.steps / dt, 1),
        "unit": "records*sweeps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": f"synthetic {a.source}",
        "config": {"model": f"oni-suspicious-connects-{a.source}-lda", "topics": a.topics, "global_batch": su.n_total,
                   "seq_len": 2 if a.source == "flow" else 1, "parallelism": f"dp{world}"},
        "step": f"one Gibbs sweep (sweeps {a.warmup + 1}..{a.warmup + a.steps} after init)",
        "gibbs_iters_per_sec": round(a.steps / dt, 3),
        "tokens_per_sec": round(tokens * a.steps / dt, 1),
        "tokens": tokens,
        "vocab": int(su.vocab.numel()),
        "setup_s": round(setup_s, 2),
        "allreduce_ms_per_sweep": model.allreduce_ms_per_sweep(),
        "allreduce_bytes_per_sweep": model.allreduce_bytes_per_sweep(),
    }


if __name__ == "__main__":
    sys.exit(main())
