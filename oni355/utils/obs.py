"""Observability: stage timers (HIP-event backed on device), roctx ranges, JSON-lines metrics
(SURVEY.md §5.1 / §5.5). The reference wrapped ml_ops.sh steps in ``time`` and relied on Spark UI
and lda-c's printed likelihoods; here every run appends one structured record to metrics.jsonl.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time

_roctx = None
_roctx_lock = threading.Lock()


def _load_roctx():
    global _roctx
    with _roctx_lock:
        if _roctx is None:
            # the rocprofiler-sdk roctx first: rocprofv3 --marker-trace intercepts that one
            for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                         "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePop.argtypes = []
                    _roctx = lib
                    break
                except OSError:
                    continue
            if _roctx is None:
                _roctx = False
    return _roctx


@contextlib.contextmanager
def range_(name: str):
    """roctx range (visible in rocprofv3 --marker-trace); no-op if roctx is unavailable."""
    lib = _load_roctx() if os.environ.get("ONI_ROCTX", "1") == "1" else False
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class StageTimer:
    """Per-stage timer used by every pipeline (oni355.pipeline.*): host wall time of each stage
    plus, on a GPU, its device time from HIP events recorded on the current stream -- so stages
    need no host synchronisation between them. :meth:`summary` gives ``<stage>_s`` (host wall)
    and ``<stage>_dev_s`` (device) entries; each stage is also a roctx range."""

    def __init__(self, device=None):
        import torch
        self.device = torch.device(device) if device is not None else None
        self.wall: dict[str, float] = {}
        self._events: list = []

    @contextlib.contextmanager
    def stage(self, name: str):
        import torch
        use_ev = self.device is not None and self.device.type == "cuda"
        if use_ev:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        t0 = time.perf_counter()
        with range_(name):
            yield
        if use_ev:
            e1.record()
            self._events.append((name, e0, e1))
        self.wall[name] = self.wall.get(name, 0.0) + time.perf_counter() - t0

    def device_ms(self) -> dict[str, float]:
        import torch
        if self._events:
            torch.cuda.synchronize(self.device)
        out: dict[str, float] = {}
        for name, e0, e1 in self._events:
            out[name] = out.get(name, 0.0) + e0.elapsed_time(e1)
        return out

    def summary(self) -> dict[str, float]:
        """``<stage>_s`` host wall seconds and ``<stage>_dev_s`` device seconds (synchronises)."""
        out = {f"{k}_s": v for k, v in self.wall.items()}
        for k, ms in self.device_ms().items():
            out[f"{k}_dev_s"] = ms / 1e3
        return out


class MetricsLog:
    """Append-only JSON-lines sink."""

    def __init__(self, path: str):
        self.path = path
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)

    def write(self, rec: dict) -> None:
        rec = {"ts": time.time(), **rec}
        with open(self.path, "a") as f:
            f.write(json.dumps(rec, default=_default) + "\n")


def _default(o):
    try:
        import numpy as np
        if isinstance(o, np.generic):
            return o.item()
        if isinstance(o, np.ndarray):
            return o.tolist()
    except ImportError:  # pragma: no cover
        pass
    return str(o)


def traced(name: str):
    """Decorator: run the function inside a roctx range ``name`` (rocprofv3 --marker-trace)."""
    import functools

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **kw):
            with range_(name):
                return fn(*a, **kw)
        return wrapper
    return deco


def heartbeat_from_env(var: str = "ONI_HEARTBEAT_S", tag: str = "heartbeat") -> bool:
    """With ``$ONI_HEARTBEAT_S`` = N, a daemon thread prints one elapsed-time line to stderr every N
    seconds: long host-side setups (1B-event synthetic days) show progress to a hang watchdog
    without the frame walking of :func:`stack_dumps_from_env`."""
    try:
        every = float(os.environ.get(var, "0") or 0)
    except ValueError:
        every = 0.0
    if every <= 0:
        return False
    import sys
    import threading
    t0 = time.perf_counter()

    def beat():
        while True:
            time.sleep(every)
            print(f"[{tag}] {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True, name="oni-heartbeat").start()
    return True


def stack_dumps_from_env(var: str = "ONI_STACK_DUMP_S") -> bool:
    """Hang diagnosis: with ``$ONI_STACK_DUMP_S`` = N, dump every thread's Python stack to stderr
    every N seconds (faulthandler), so a stalled run names the call it is stuck in.

    Diagnostic runs only: the dump walks the other threads' frames without holding the GIL and
    can crash a busy interpreter (seen once, mid list-comprehension, after ~6 dumps)."""
    try:
        every = float(os.environ.get(var, "0") or 0)
    except ValueError:
        every = 0.0
    if every <= 0:
        return False
    import faulthandler
    faulthandler.dump_traceback_later(every, repeat=True)
    return True
