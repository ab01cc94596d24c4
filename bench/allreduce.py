#!/usr/bin/env python3
"""RCCL all-reduce bandwidth over xGMI for the per-sweep Δn_wk payload.

Sweeps int32 SUM all-reduces from 64 KiB to --max-mb MiB (the flow config's Δ is V·KS·4 ≈ 0.4 MB,
DNS/proxy at V ≈ 10⁶ and K = 50/100 reach 0.2-0.4 GB) and prints one JSON line per size with the
max-over-ranks time, algorithm bandwidth (bytes / t) and ring bus bandwidth (2(N-1)/N · bytes / t),
so the Δ payload can be priced against the per-link bound (7 xGMI links × ≈153 GB/s per GPU).

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/allreduce.py
  python bench/allreduce.py --device cpu            # gloo, plumbing only
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
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--min-kb", type=int, default=64)
    ap.add_argument("--max-mb", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args(argv)
    import torch

    from oni355.parallel import comm as pc
    comm = pc.init_from_env(a.device)
    dev = comm.device
    n = comm.world

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    size = a.min_kb * 1024
    while size <= a.max_mb * 1024 * 1024:
        t = torch.ones(size // 4, dtype=torch.int32, device=dev)
        for _ in range(a.warmup):
            comm.allreduce_(t)
        sync()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            comm.allreduce_(t)
        sync()
        dt = comm.allreduce_scalar((time.perf_counter() - t0) / a.iters, "max")
        ok = int(t[0].item()) == n ** (a.warmup + a.iters) if n > 1 else True
        if comm.rank == 0:
            alg = size / dt
            print(json.dumps({"bytes": size, "ranks": n, "us": round(dt * 1e6, 2), "algbw_GBps": round(alg / 1e9, 3),
                              "busbw_GBps": round(alg * 2 * (n - 1) / max(n, 1) / 1e9, 3), "ok": ok}), flush=True)
        del t
        size *= 4
    pc.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
