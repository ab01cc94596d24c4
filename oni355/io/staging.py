"""Host → HBM column upload through the native pinned staging ring (csrc/kernels/stage.hip).

SURVEY.md §2.4 P3/P7 (partition-parallel ingest, stage overlap): decoded host columns go to the
GPU through a ring of pinned buffers filled by several host threads while the DMA engine drains
the previous chunk; :func:`upload` returns once the last chunk is queued on torch's current
stream, so the wordify / quantile kernels launched next are ordered after the copies and the host
moves on to the next column (or the next decoded part) at once. The reference's equivalent hop is
HDFS → Spark executors → lda-c corpus files shipped to MPI nodes.

``ONI_STAGED_H2D``: ``0`` plain ``tensor.to(device)`` (default), ``1`` ring, ``reg`` pin the
source in place and DMA it directly. Measured on MI355X (``bench/h2d.py``, 550 MB of flow columns,
``profiles/r1_h2d_staging.jsonl``): every path is PCIe-link bound, plain 9.98 ms (55.1 GB/s),
registered 9.93 ms (55.4 GB/s), ring 10.63 ms (51.7 GB/s at 32 MB chunks x 16 threads; 27-31 GB/s
at 4-8 MB chunks: the host memcpy into pinned memory is the ring's bottleneck). ROCm's own pageable
copy path already reaches the link rate, so plain stays the default; the ring and the registered
path are kept as measured options.
CPU targets return the host tensor itself.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import threading

import numpy as np
import torch

from ..ops import _lib

vp, i64 = C.c_void_p, C.c_int64
_lib.register_optional("oni_stager_create", [i64, C.c_int, C.c_int, C.POINTER(C.c_void_p)])
_lib.register_optional("oni_stager_upload", [vp, vp, vp, i64, vp])
_lib.register_optional("oni_stager_sync", [vp])
_lib.register_optional("oni_stager_stats", [vp, vp])
_lib.register_optional("oni_stager_destroy", [vp])
_lib.register_optional("oni_h2d_registered", [vp, vp, i64, vp])

CHUNK_BYTES = int(os.environ.get("ONI_STAGE_CHUNK_MB", "32")) << 20
N_BUF = 3
THREADS = int(os.environ.get("ONI_STAGE_THREADS", "16"))

_lock = threading.Lock()
_handle: C.c_void_p | None = None


def mode() -> str:
    m = os.environ.get("ONI_STAGED_H2D", "0")
    return {"0": "plain", "1": "ring", "reg": "reg"}.get(m, "plain")


def _stager() -> C.c_void_p:
    global _handle
    with _lock:
        if _handle is None:
            h = C.c_void_p()
            _lib.check(_lib.lib().oni_stager_create(CHUNK_BYTES, N_BUF, THREADS, C.byref(h)), "oni_stager_create")
            _handle = h
            atexit.register(_destroy)
        return _handle


def _destroy() -> None:
    global _handle
    with _lock:
        if _handle is not None:
            _lib.lib().oni_stager_destroy(_handle)
            _handle = None


def upload_tensor(t: torch.Tensor, device) -> torch.Tensor:
    """Copy CPU tensor ``t`` to ``device`` (same dtype and shape) by the selected :func:`mode`."""
    device = torch.device(device)
    m = mode()
    if device.type != "cuda" or m == "plain":
        return t.to(device)
    src = t.contiguous()
    out = torch.empty(src.shape, dtype=src.dtype, device=device)
    nbytes = src.numel() * src.element_size()
    if nbytes:
        with torch.cuda.device(device):
            if m == "reg":
                _lib.check(_lib.lib().oni_h2d_registered(src.data_ptr(), out.data_ptr(), nbytes, _lib.stream()),
                           "oni_h2d_registered")
            else:
                _lib.check(_lib.lib().oni_stager_upload(_stager(), src.data_ptr(), out.data_ptr(), nbytes,
                                                        _lib.stream()), "oni_stager_upload")
    return out


def upload(a, device, dtype: torch.dtype | None = None) -> torch.Tensor:
    """NumPy array (or CPU tensor) → device tensor; ``dtype`` converts on the host first."""
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return upload_tensor(t, device)


def sync() -> None:
    """Block until every queued chunk has landed."""
    if _handle is not None:
        _lib.check(_lib.lib().oni_stager_sync(_handle), "oni_stager_sync")


def stats() -> dict:
    """Bytes and chunks moved through the ring by this process."""
    if _handle is None:
        return {"bytes": 0, "chunks": 0}
    out = (C.c_int64 * 2)()
    _lib.check(_lib.lib().oni_stager_stats(_handle, out), "oni_stager_stats")
    return {"bytes": int(out[0]), "chunks": int(out[1])}


class Prefetcher:
    """Double-buffered host → HBM upload of the NEXT day's device columns on a dedicated copy
    stream, overlapping the current day's compute (SURVEY.md §2.4 P7 stage overlap).

    A loader that owns pinned host buffers (:meth:`pin`, done once per buffer) submits day k+1
    while day k trains; :meth:`take` makes the compute stream wait for the copies (an event, no
    host sync) and hands the tensors over. Each submitted day is a full upload; only its timing
    overlaps. ``copy_ms()`` reports the device time of the last completed upload."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self._pending = None
        self._last = None

    @staticmethod
    def pin(cols: dict, specs: dict) -> dict:
        """Page-locked host copies of ``cols`` converted to the device dtypes of ``specs``."""
        out = {}
        for name, dt in specs.items():
            a = np.asarray(cols[name])
            if a.dtype == np.uint32:
                a = a.view(np.int32)
            t = torch.from_numpy(np.ascontiguousarray(a)).to(dt)
            out[name] = t.pin_memory()
        return out

    def submit(self, pinned: dict) -> None:
        if self._pending is not None:
            raise RuntimeError("Prefetcher: take() the pending upload first")
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(self.stream)
            out = {k: t.to(self.device, non_blocking=True) for k, t in pinned.items()}
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(self.stream)
        self._pending = (out, e0, e1)

    def take(self) -> dict:
        out, e0, e1 = self._pending
        self._pending = None
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(e1)
        for t in out.values():
            t.record_stream(cur)  # allocated on the copy stream, consumed and freed on the compute stream
        self._last = (e0, e1)
        return out

    def copy_ms(self) -> float | None:
        if self._last is None:
            return None
        self._last[1].synchronize()
        return self._last[0].elapsed_time(self._last[1])
