"""``oni-ml`` -- the ``ml_ops.sh YYYYMMDD {flow,dns,proxy} [TOL] [MAXRESULTS]`` equivalent.

Reference ([U-M]): ml_ops.sh sources /etc/duxbay.conf, removes the day's HDFS
output, resolves ``${LPATH}/${DSOURCE}_scores.csv`` as feedback, runs the Spark job (pre-LDA →
mpiexec lda est → post-LDA) and getmerges ``${LPATH}/${DSOURCE}_results.csv``.

Here: one process per GPU (``--gpus N`` re-launches itself under torch.distributed.run over
RCCL), data from the columnar store (``--data-root``), raw files (``--input``: flow CSV / nfcapd,
pcap, proxy log) or the synthetic generators (``--synthetic N``); results go to
``<LPATH>/<source>/<YYYYMMDD>/<source>_results.csv`` (+ ``metrics.jsonl``, optional lda-c files).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="oni-ml", description="MI355X suspicious-connects (ONI oni-ml equivalent)")
    ap.add_argument("date", help="YYYYMMDD, a range YYYYMMDD-YYYYMMDD or a comma list (several days: one process "
                                 "scores them back to back, each day's store read + pin + upload overlapping the "
                                 "previous day's GPU work)")
    ap.add_argument("source", choices=["flow", "dns", "proxy"])
    ap.add_argument("tol", nargs="?", type=float, default=None, help="keep scores below TOL")
    ap.add_argument("maxresults", nargs="?", type=int, default=None)
    ap.add_argument("--config", default=os.environ.get("ONI_CONFIG", "/etc/duxbay.conf"))
    ap.add_argument("--device", default=None, choices=["cuda", "cpu"])
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (one process each); default PROCESS_COUNT")
    ap.add_argument("--data-root", default=None)
    ap.add_argument("--input", action="append", default=[], help="raw input file/glob (repeatable)")
    ap.add_argument("--synthetic", type=int, default=0, help="generate N synthetic events instead of loading")
    ap.add_argument("--topics", type=int, default=None)
    ap.add_argument("--sweeps", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--alpha", type=float, default=None)
    ap.add_argument("--beta", type=float, default=None)
    ap.add_argument("--chunk-len", type=int, default=None)
    ap.add_argument("--dupfactor", type=int, default=None)
    ap.add_argument("--user-domain", default=None)
    ap.add_argument("--top-domains", default=None, help="top-1M list (rank,domain CSV)")
    ap.add_argument("--lpath", default=None)
    ap.add_argument("--feedback", default=None, help="scores CSV (default <LPATH>/<source>_scores.csv)")
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--ckpt-every", type=int, default=None)
    ap.add_argument("--eval-every", type=int, default=None)
    ap.add_argument("--ldac-out", default=None, help="write lda-c files (final.beta/gamma/other, likelihood.dat)")
    ap.add_argument("--ldac-lag", type=int, default=0, help="also write lda-c NNN.* snapshots every N sweeps")
    ap.add_argument("--burnin", type=int, default=None, help="sweeps before the likelihood trace / snapshots")
    ap.add_argument("--max-restarts", type=int, default=0,
                    help="supervise the run: after a failure (crash, watchdog exit, numerical fault) start a "
                         "fresh child process that resumes from the last checkpoint, up to R times")
    ap.add_argument("--follow", action="store_true",
                    help="after the given day(s), keep scoring every later day the store completes (_SUCCESS)")
    ap.add_argument("--poll", type=float, default=5.0, help="--follow: seconds between store scans")
    ap.add_argument("--idle-exit", type=float, default=3600.0,
                    help="--follow: stop after this many seconds without a new complete day")
    ap.add_argument("--max-days", type=int, default=0, help="stop after N days (0: no limit)")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--service", metavar="SOCKET",
                    help="forward this run to a warm oni-mld service on SOCKET (env ONI_MLD_SOCKET); runs locally "
                         "when none answers")
    return ap


def _relaunch(n: int, argv: list[str]) -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "oni355.cli.ml", *argv, "--gpus", str(n)]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def _strip_opt(argv: list[str], name: str) -> list[str]:
    out, skip = [], False
    for i, x in enumerate(argv):
        if skip:
            skip = False
            continue
        if x == name:
            skip = True
            continue
        if x.startswith(name + "="):
            continue
        out.append(x)
    return out


def supervise(a, argv: list[str], cfg) -> int:
    """``--max-restarts R``: run the job as a child process; when it fails, start a FRESH child
    (never an exec, nothing here touches the GPU) that resumes from the last checkpoint, up to R
    times -- the role Spark/YARN task retry played for oni-ml. Checkpoints go to
    ``--ckpt-dir`` (default ``<LPATH>/<source>/<date>/.ckpt``, every ``--ckpt-every`` sweeps,
    default 20). Each child sees ``ONI_RESTART_COUNT`` (the attempt number), which
    ``ONI_FAULT=...,attempt:A`` uses to fail only a given attempt."""
    import shutil
    child = _strip_opt(argv, "--max-restarts")
    own_dir = a.ckpt_dir is None
    ck = a.ckpt_dir or os.path.join(cfg.LPATH, a.source, a.date, ".ckpt")
    if own_dir:
        shutil.rmtree(ck, ignore_errors=True)
        child += ["--ckpt-dir", ck]
    if a.ckpt_every is None and cfg.CKPT_EVERY <= 0:
        child += ["--ckpt-every", "20"]
    rc = 1
    for attempt in range(a.max_restarts + 1):
        env = dict(os.environ, ONI_SUPERVISED="1", ONI_RESTART_COUNT=str(attempt))
        rc = subprocess.run([sys.executable, "-m", "oni355.cli.ml", *child], env=env).returncode
        if rc == 0:
            break
        print(f"[oni-ml] attempt {attempt} failed (exit {rc})"
              + ("; restarting from the last checkpoint" if attempt < a.max_restarts else "; giving up"),
              file=sys.stderr, flush=True)
    if rc == 0 and own_dir:
        shutil.rmtree(ck, ignore_errors=True)
    return rc


def _expand(inputs: list[str]) -> list[str]:
    out = []
    for p in inputs:
        if os.path.isdir(p):
            out += sorted(q for q in glob.glob(os.path.join(p, "*")) if os.path.isfile(q))
        else:
            out += sorted(glob.glob(p)) or [p]
    return out


def _concat(parts: list[dict]) -> dict:
    from ..store.columnar import StringColumn
    if len(parts) == 1:
        return parts[0]
    out = {}
    for k in parts[0]:
        if k.startswith("_"):
            continue
        v = [p[k] for p in parts]
        out[k] = StringColumn.concat(v) if isinstance(v[0], StringColumn) else np.concatenate(v)
    return out


def _slice(cols: dict, lo: int, hi: int) -> dict:
    from ..store.columnar import StringColumn
    return {k: (v.slice(lo, hi) if isinstance(v, StringColumn) else v[lo:hi]) for k, v in cols.items() if not k.startswith("_")}


def load_events(a, cfg, source: str, rank: int, world: int) -> tuple[dict, int, int]:
    """Returns (columns of this rank's rows, global row offset, global row count)."""
    from ..io import decoders
    from ..store import columnar
    if a.synthetic:
        per = a.synthetic // world
        lo = rank * per
        n = a.synthetic - lo if rank == world - 1 else per
        if source == "flow":
            from ..synth.flow import generate_flows
            day = generate_flows(a.synthetic, seed=cfg.SEED & 0xFFFF)
            return _slice(day.cols, lo, lo + n), lo, a.synthetic
        if source == "dns":
            from ..synth.dns import generate_dns
            day = generate_dns(a.synthetic, seed=cfg.SEED & 0xFFFF, user_domain=cfg.USER_DOMAIN or "intel")
            return _slice(day.cols, lo, lo + n), lo, a.synthetic
        from ..synth.proxy import generate_proxy
        day = generate_proxy(a.synthetic, seed=cfg.SEED & 0xFFFF)
        return _slice(day.cols, lo, lo + n), lo, a.synthetic
    files = _expand(a.input)
    if files:
        parts = []
        for f in files:
            if source == "flow":
                if f.endswith(".csv") or f.endswith(".txt"):
                    parts.append(decoders.read_flow_csv(f)[0])
                else:
                    from ..io import nfcapd
                    parts.append(nfcapd.read_nfcapd(f))
            elif source == "dns":
                parts.append(decoders.read_pcap_dns(f))
            else:
                parts.append(decoders.read_proxy_log(f))
        cols = _concat(parts)
        n = len(cols["sip" if source == "flow" else ("ip_dst" if source == "dns" else "clientip")])
        per = n // world
        lo = rank * per
        hi = n if rank == world - 1 else lo + per
        return _slice(cols, lo, hi), lo, n
    root = a.data_root or cfg.DATA_ROOT
    n = columnar.rows(root, source, a.date)
    per = n // world
    lo = rank * per
    hi = n if rank == world - 1 else lo + per
    return columnar.read_day(root, source, a.date, row_range=(lo, hi)), lo, n


def _service_socket(argv: list[str]) -> tuple[str | None, list[str]]:
    """``--service PATH`` / ``ONI_MLD_SOCKET``: the resident service (oni355.cli.service) to forward
    to; returns (path or None, argv without the option)."""
    path = os.environ.get("ONI_MLD_SOCKET") or None
    out, it = [], iter(range(len(argv)))
    for i in it:
        if argv[i] == "--service" and i + 1 < len(argv):
            path = argv[i + 1]
            next(it, None)
        elif argv[i].startswith("--service="):
            path = argv[i].split("=", 1)[1]
        else:
            out.append(argv[i])
    return path, out


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    svc, argv = _service_socket(argv)
    if svc and os.environ.get("ONI_MLD_INSIDE") != "1":
        # a warm service answers: the day runs there (nothing here has imported torch yet)
        from .service import forward
        rc = forward(svc, argv)
        if rc is not None:
            return rc
    a = build_parser().parse_args(argv)
    from ..config import load_config
    cfg = load_config(a.config if a.config and os.path.exists(a.config) else None,
                      TOPIC_COUNT=a.topics, SWEEPS=a.sweeps, SEED=a.seed, BETA=a.beta, CHUNK_LEN=a.chunk_len,
                      DUPFACTOR=a.dupfactor, USER_DOMAIN=a.user_domain, LPATH=a.lpath, EVAL_EVERY=a.eval_every,
                      CKPT_EVERY=a.ckpt_every, TOP_DOMAINS=a.top_domains, TOL=a.tol, MAXRESULTS=a.maxresults,
                      ALPHA=a.alpha, BURNIN=a.burnin)
    inside = os.environ.get("ONI_MLD_INSIDE") == "1"
    if a.max_restarts > 0 and os.environ.get("ONI_SUPERVISED") != "1":
        if inside:
            # the supervisor's children would write to the service's stdout, not the client's
            from .service import RunLocally
            raise RunLocally("a supervised run (--max-restarts) starts child processes")
        return supervise(a, argv, cfg)
    if cfg.PUBLIC_SUFFIX:
        os.environ["ONI_PUBLIC_SUFFIX"] = cfg.PUBLIC_SUFFIX  # read by oni355.ref.psl.default_rules
    gpus = a.gpus if a.gpus is not None else cfg.PROCESS_COUNT
    if gpus > 1 and "WORLD_SIZE" not in os.environ:
        if inside:
            from .service import RunLocally
            raise RunLocally(f"{gpus} GPUs: one process per GPU")
        return _relaunch(gpus, argv)

    import torch

    from ..io import results as rio
    from ..parallel import comm as pc
    from ..utils.obs import MetricsLog

    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    comm = pc.init_from_env(device)
    rank, world = comm.rank, comm.world
    log = (lambda m: None) if (a.quiet or rank) else (lambda m: print(f"[oni-ml] {m}", file=sys.stderr, flush=True))
    from ..pipeline.daily import parse_dates
    dates = parse_dates(a.date)
    if len(dates) > 1 or a.follow:
        return _main_days(a, cfg, comm, device, dates, log)
    t0 = time.perf_counter()
    cols, row_off, n_total = load_events(a, cfg, a.source, rank, world)
    t_load = time.perf_counter() - t0
    log(f"{a.source} {a.date}: {n_total} events, {world} rank(s) on {device}")
    fb_path = a.feedback or rio.scores_path(cfg.LPATH, a.source)
    from ..oa import feedback as fbm
    fb = fbm.load_feedback(fb_path, a.source) if os.path.exists(fb_path) else None
    if fb is not None:
        log(f"feedback: {len(next(iter(fb.values())))} sev=3 rows from {fb_path} (x{cfg.DUPFACTOR})")
    ckpt = None
    if a.ckpt_dir:
        from ..utils.checkpoint import Checkpointer
        ckpt = Checkpointer(a.ckpt_dir, cfg.CKPT_EVERY, comm)
    top = None
    if cfg.TOP_DOMAINS:
        from ..pipeline.dns import load_top_domains
        top = load_top_domains(cfg.TOP_DOMAINS)
    alpha = cfg.ALPHA if cfg.ALPHA > 0 else None
    common_kw = dict(K=cfg.TOPIC_COUNT, sweeps=cfg.SWEEPS, tol=cfg.TOL, maxresults=cfg.MAXRESULTS, alpha=alpha,
                     beta=cfg.BETA, seed=cfg.SEED, chunk_len=cfg.CHUNK_LEN, device=device, comm=comm, feedback=fb,
                     dupfactor=cfg.DUPFACTOR, row_offset=row_off, eval_every=cfg.EVAL_EVERY, burnin=cfg.BURNIN,
                     ckpt=ckpt, log=log)
    if a.ldac_out and a.ldac_lag > 0:
        common_kw.update(ldac_dir=os.path.join(a.ldac_out, f"rank{rank}") if world > 1 else a.ldac_out,
                         ldac_lag=a.ldac_lag)
    if a.source == "flow":
        from ..pipeline.flow import run_flow
        res = run_flow(cols, **common_kw)
    elif a.source == "dns":
        from ..pipeline.dns import run_dns
        res = run_dns(cols, top_domains=top, user_domain=cfg.USER_DOMAIN, **common_kw)
    else:
        from ..pipeline.proxy import run_proxy
        res = run_proxy(cols, top_domains=top, **common_kw)
    rendered = rio.render_result(a.source, cols, res, row_off, comm)
    out = None
    if rank == 0:
        from .. import schema
        out = rio.write_rendered(rio.results_path(cfg.LPATH, a.source, a.date), schema.result_columns(a.source),
                                 rendered)
        m = MetricsLog(os.path.join(os.path.dirname(out), "metrics.jsonl"))
        m.write({"event": "oni-ml", "source": a.source, "date": a.date, "events": n_total, "ranks": world,
                 "device": device, "load_s": t_load, **{k: v for k, v in res.timings.items()},
                 **{k: v for k, v in res.stats.items() if isinstance(v, (int, float, str)) or v is None}})
        log(f"wrote {len(rendered)} rows -> {out}")
    if a.ldac_out:
        from ..io import ldac
        d = os.path.join(a.ldac_out, f"rank{rank}") if world > 1 else a.ldac_out
        ldac.export_gibbs(d, res.lda.model)
    comm.barrier()
    pc.shutdown()
    if rank == 0 and not a.quiet:
        print(json.dumps({"results": out, "rows": len(rendered), "timings": res.timings}))
    return 0


def _main_days(a, cfg, comm, device, dates: list[str], log) -> int:
    """Several days (a range, a list, ``--follow``) from the columnar store in one process: the
    day pipeline of oni355.pipeline.daily (store read + pin + upload of day k+1 overlap day k)."""
    from ..io import results as rio
    from ..parallel import comm as pc
    from ..pipeline.daily import run_days
    if a.synthetic or a.input:
        raise SystemExit("oni-ml: several days / --follow read the columnar store (--data-root), not --synthetic/--input")
    if a.ckpt_dir or a.ldac_out:
        raise SystemExit("oni-ml: --ckpt-dir / --ldac-out apply to single-day runs")
    root = a.data_root or cfg.DATA_ROOT
    top = None
    if cfg.TOP_DOMAINS:
        from ..pipeline.dns import load_top_domains
        top = load_top_domains(cfg.TOP_DOMAINS)
    alpha = cfg.ALPHA if cfg.ALPHA > 0 else None
    kw = dict(K=cfg.TOPIC_COUNT, sweeps=cfg.SWEEPS, tol=cfg.TOL, maxresults=cfg.MAXRESULTS, alpha=alpha,
              beta=cfg.BETA, seed=cfg.SEED, chunk_len=cfg.CHUNK_LEN, device=device, dupfactor=cfg.DUPFACTOR,
              eval_every=cfg.EVAL_EVERY, burnin=cfg.BURNIN, log=log)
    if a.source == "dns":
        kw.update(top_domains=top, user_domain=cfg.USER_DOMAIN)
    elif a.source == "proxy":
        kw.update(top_domains=top)
    t0 = time.perf_counter()
    recs = run_days(a.source, dates, root, cfg.LPATH, comm, kw, device, follow=a.follow, poll_s=a.poll,
                    idle_exit_s=a.idle_exit, max_days=a.max_days,
                    feedback_path=a.feedback or rio.scores_path(cfg.LPATH, a.source), log=log)
    wall = time.perf_counter() - t0
    comm.barrier()
    pc.shutdown()
    if comm.rank == 0 and not a.quiet:
        print(json.dumps({"days": [r["date"] for r in recs], "wall_s": round(wall, 3),
                          "s_per_day": round(wall / max(len(recs), 1), 4),
                          "events": int(sum(r["events"] for r in recs))}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
