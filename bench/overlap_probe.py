"""Which work on the compute stream waits behind a bulk H2D copy on a copy stream?

A 550 MB pinned upload (one flow day) runs on its own stream; meanwhile the compute stream does one
kind of work and we time it (host wall and HIP events). Kinds: plain kernels, a HIP-graph replay of
the same kernels, a small pageable H2D, a small D2H, a D2D copy, a 1-rank RCCL all-reduce.

    python bench/overlap_probe.py [--mb 550]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=550)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    import torch.distributed as dist
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    host = torch.empty(a.mb << 20, dtype=torch.uint8).pin_memory()
    dst = torch.empty_like(host, device=dev)
    cs = torch.cuda.Stream(dev)
    x = torch.randn(1 << 22, device=dev)
    small = torch.arange(4096, dtype=torch.int64)
    small_d = torch.zeros(4096, dtype=torch.int64, device=dev)
    red = torch.ones(1 << 16, dtype=torch.int32, device=dev)

    def kernels():
        for _ in range(50):
            x.mul_(1.0001)

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        kernels()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        kernels()
    kinds = {
        "kernels": kernels,
        "graph": g.replay,
        "h2d_small_pageable": lambda: small_d.copy_(small),
        "d2h_small": lambda: small_d.cpu(),
        "d2d": lambda: x.clone(),
        "rccl_allreduce": lambda: dist.all_reduce(red),
        "full_fill": lambda: torch.full((1,), 3, device=dev),
    }
    from oni355.io import staging
    hp = torch.cuda.Stream(dev, priority=-1)
    side = torch.cuda.Stream(dev)
    busy_kinds = {
        "dma": lambda: (cs.wait_stream(torch.cuda.current_stream()), _on(cs, lambda: dst.copy_(host, non_blocking=True))),
        "pull": lambda: (cs.wait_stream(torch.cuda.current_stream()), staging.pull_upload(host, dev, cs)),
        "pull_hiprio": lambda: (hp.wait_stream(torch.cuda.current_stream()), staging.pull_upload(host, dev, hp)),
    }
    out = {}
    for bname, busy_fn in busy_kinds.items():
        for cur in ("default", "side"):
            for name, fn in kinds.items():
                ctx = torch.cuda.stream(side) if cur == "side" else _null()
                with ctx:
                    res = _measure(fn, busy_fn)
                out[f"{bname}/{cur}/{name}"] = res
                print(bname, cur, name, res, flush=True)
    print(json.dumps(out))
    dist.destroy_process_group()


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _on(stream, fn):
    with torch.cuda.stream(stream):
        return fn()


def _measure(fn, busy_fn):
    res = {}
    for busy in (False, True):
        fn()
        torch.cuda.synchronize()
        if busy:
            busy_fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        res["busy" if busy else "idle"] = round((time.perf_counter() - t0) * 1e3, 3)
        torch.cuda.synchronize()
    return res


if __name__ == "__main__":
    main()
