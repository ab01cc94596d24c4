"""Which part of the data-parallel featurize stage waits behind the Prefetcher's bulk upload?

Each variant is run once idle and once right after a 550 MB upload was queued on the copy
stream; host wall times are printed (a variant that waits shows ≈ the upload time).

    MASTER_ADDR=127.0.0.1 MASTER_PORT=29563 python bench/featurize_probe.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    nodist = os.environ.get("PROBE_NODIST") == "1"  # no process group at all (the world-1 bench)
    os.environ["ONI_FORCE_DIST"] = "0" if nodist else "1"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29563")
    from oni355 import ops
    from oni355.io.staging import Prefetcher
    from oni355.parallel.comm import init_from_env
    from oni355.ref import spec
    pf = None
    if os.environ.get("PROBE_PF_FIRST") == "1":  # copy stream created before the process group
        torch.cuda.set_device(0)
        pf = Prefetcher(torch.device("cuda", 0))
    comm = init_from_env("cuda")
    dev = comm.device
    host = {"x": torch.empty(550 << 20, dtype=torch.uint8).pin_memory()}
    pf = pf or Prefetcher(dev)
    keys = torch.randint(0, 2**31 - 1, (25_000_000,), dtype=torch.int32, device=dev)
    small = torch.zeros(2048, dtype=torch.int32, device=dev)
    hist = torch.zeros(2048, dtype=torch.int32, device=dev)

    variants = {
        "d2h_8KB": lambda: small.cpu(),
        "item": lambda: small[0].item(),
        "allreduce_np_scalar": lambda: comm.allreduce_np(np.array([5], np.int64)),
        "allreduce_np_devtensor": lambda: comm.allreduce_np(hist.to(torch.int64)),
        "allreduce_scalar": lambda: comm.allreduce_scalar(1.0),
        "h2d_from_numpy": lambda: torch.from_numpy(np.arange(16, dtype=np.int32)).to(dev),
        "quantile_local": lambda: ops.quantile_cuts(keys, spec.DECILES),
        "quantile_dist": lambda: ops.quantile_cuts(keys, spec.DECILES, comm.allreduce_np, keys.numel()),
    }
    if nodist:
        variants = {k: v for k, v in variants.items() if "allreduce" not in k and k != "quantile_dist"}
    for name, fn in variants.items():
        res = {}
        for busy in (False, True):
            fn()
            torch.cuda.synchronize()
            if busy:
                pf.submit(host)
            t0 = time.perf_counter()
            fn()
            ev = torch.cuda.Event()
            ev.record()
            ev.synchronize()  # this stream only (a device-wide sync would include the upload)
            t1 = time.perf_counter()
            res["busy" if busy else "idle"] = round((t1 - t0) * 1e3, 3)
            if busy:
                pf.take()
                torch.cuda.synchronize()
        print(name, res, flush=True)


if __name__ == "__main__":
    main()
