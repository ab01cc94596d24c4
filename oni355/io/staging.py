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
import warnings

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
_lib.register_optional("oni_h2d_pull", [vp, vp, i64, C.c_int, vp])
_lib.register_optional("oni_d2h_push", [vp, vp, i64, vp])

# Prefetcher uploads: "dma" (hipMemcpyAsync) or "pull" (CUs read the pinned host buffers and the
# DMA engine stays free). Measured (bench/overlap_probe.py, profiles/r2_copy_overlap_probe.txt):
# behind a 550 MB DMA upload, kernels / graph replays / D2D / RCCL on the compute stream run at
# full speed and only small H2D/D2H transfers wait; behind the pull kernel every kernel waits.
# So "dma" is the default and the run avoids DMA transfers while an upload is in flight.
PREFETCH_COPY = os.environ.get("ONI_PREFETCH_COPY", "dma")
PULL_BLOCKS = int(os.environ.get("ONI_PULL_BLOCKS", "64"))

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
    if isinstance(a, torch.Tensor):
        t = a
    else:
        a = np.ascontiguousarray(a)
        if a.flags.writeable:
            t = torch.from_numpy(a)
        else:
            # a read-only store memmap: wrapped without a copy, and this tensor is only ever the
            # source of the device copy (or of a dtype conversion, which allocates), never written
            with warnings.catch_warnings():
                warnings.filterwarnings("ignore", message="The given NumPy array is not writable")
                t = torch.from_numpy(a)
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return upload_tensor(t, device)


def pull_upload(src: torch.Tensor, device, stream=None, blocks: int = PULL_BLOCKS) -> torch.Tensor:
    """Pinned CPU tensor → device tensor copied by a kernel (``oni_h2d_pull``) on ``stream``
    (default: the current stream), not by the DMA engine. Falls back to a non-blocking DMA copy
    when the source is not device-visible pinned memory."""
    device = torch.device(device)
    out = torch.empty(src.shape, dtype=src.dtype, device=device)
    nbytes = src.numel() * src.element_size()
    if nbytes == 0:
        return out
    st = stream if stream is not None else torch.cuda.current_stream(device)
    rc = _lib.lib().oni_h2d_pull(src.data_ptr(), out.data_ptr(), nbytes, int(blocks), st.cuda_stream) \
        if src.is_pinned() else -1
    if rc != 0:
        with torch.cuda.stream(st):
            out.copy_(src, non_blocking=True)
    return out


def push_to_host(src: torch.Tensor, dst: torch.Tensor) -> None:
    """Queue a copy of the 4-byte-element device tensor ``src`` into the pinned CPU tensor ``dst``
    by a kernel on the current stream (``oni_d2h_push``), so a small read-back does not queue
    behind a bulk upload on the DMA engine. Read ``dst`` after an event recorded behind this call
    has completed. Falls back to a non-blocking DMA copy."""
    if src.element_size() != 4 or dst.element_size() != 4 or src.numel() != dst.numel():
        raise ValueError("push_to_host: 4-byte elements of equal count")
    src = src.contiguous()
    rc = -1
    if dst.is_pinned() and dst.is_contiguous():
        rc = _lib.lib().oni_d2h_push(src.data_ptr(), dst.data_ptr(), src.numel(),
                                     torch.cuda.current_stream(src.device).cuda_stream)
    if rc != 0:
        dst.copy_(src, non_blocking=True)


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
    overlaps. ``copy_ms()`` reports the device time of the last completed upload.

    The copy stream is high priority: with a default-priority stream (and a process group
    initialised) every small read-back or upload of the day being computed -- quantile histograms,
    all-to-all counts, ``.item()`` -- waited for the whole 550 MB upload (10 ms of a forced 1-rank
    day, ``bench/featurize_probe.py``). The sampler's own polling read-back is a kernel store
    (:func:`push_to_host`) either way."""

    def __init__(self, device):
        self.device = torch.device(device)
        # a high-priority stream gets its own hardware queue: with a process group initialised, a
        # default-priority copy stream made every small H2D/D2H of the compute stream wait for the
        # whole upload (bench/featurize_probe.py: 10.2 ms → 0.06 ms per read-back)
        self.stream = torch.cuda.Stream(self.device, priority=int(os.environ.get("ONI_PREFETCH_PRIORITY", "-1")))
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

    @staticmethod
    def pin_arrays(arrays: dict) -> dict:
        """Page-locked host copies of ready-typed arrays (e.g. a pipeline's ``host_arrays``)."""
        return {k: torch.from_numpy(np.ascontiguousarray(a)).pin_memory() for k, a in arrays.items()}

    def submit(self, pinned: dict) -> None:
        if self._pending is not None:
            raise RuntimeError("Prefetcher: take() the pending upload first")
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(self.stream)
            if PREFETCH_COPY == "pull":
                out = {k: pull_upload(t, self.device, self.stream) for k, t in pinned.items()}
            else:
                out = {k: t.to(self.device, non_blocking=True) for k, t in pinned.items()}
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(self.stream)
        self._pending = (out, e0, e1)

    def last_event(self):
        """Event recorded after the pending upload's copies (a PinnedSlots slot may be reused once
        it has completed)."""
        return self._pending[2] if self._pending is not None else None

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


class PinnedSlots:
    """Reusable page-locked buffers for the multi-day loader: ``n_slots`` sets of per-column
    pinned tensors, refilled round-robin (allocating 550 MB of pinned memory per day cost more than
    the copy into it). A slot is refilled only after the upload that last read it has finished
    (``mark_used(slot, event)``). Columns are copied in parallel slices by ``threads`` workers --
    numpy releases the GIL for the copies, so the loader thread is not one memcpy stream."""

    def __init__(self, n_slots: int = 3, threads: int = 8):
        from concurrent.futures import ThreadPoolExecutor
        self.slots: list[dict] = [dict() for _ in range(n_slots)]
        self.events: list = [None] * n_slots
        self.k = 0
        self.pool = ThreadPoolExecutor(threads, thread_name_prefix="oni-pincopy")
        self.threads = threads

    def _buf(self, slot: dict, name: str, n: int, dtype: torch.dtype) -> torch.Tensor:
        t = slot.get(name)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(max(n, 1), dtype=dtype).pin_memory()
            slot[name] = t
        return t[:n]

    def fill(self, arrays: dict, dtypes: dict | None = None) -> tuple[int, dict]:
        """(slot index, pinned tensors) holding ``arrays`` (name → array-like; memmaps are read
        here), converted to ``dtypes[name]`` when given."""
        i = self.k
        self.k = (self.k + 1) % len(self.slots)
        ev = self.events[i]
        if ev is not None:
            ev.synchronize()  # the upload that last read this slot has finished
        slot = self.slots[i]
        out, futs = {}, []
        for name, a in arrays.items():
            a = np.asarray(a)
            if a.dtype == np.uint32:
                a = a.view(np.int32)
            dt = dtypes[name] if dtypes else torch.from_numpy(a[:0]).dtype
            t = self._buf(slot, name, a.shape[0], dt)
            dst = t.numpy()
            step = max(1 << 20, -(-a.shape[0] // self.threads))
            for lo in range(0, a.shape[0], step):
                futs.append(self.pool.submit(np.copyto, dst[lo:lo + step], a[lo:lo + step], "unsafe"))
            out[name] = t
        for f in futs:
            f.result()
        return i, out

    def mark_used(self, slot: int, event) -> None:
        self.events[slot] = event

    def close(self) -> None:
        self.pool.shutdown(wait=True)


class HostAhead:
    """Run a host-side producer (a decoder: pcap → columns) one item ahead on a worker thread,
    so decoding day k+1 overlaps the GPU work of day k (SURVEY.md §2.4 P7 "decode ‖ H2D ‖
    compute"). The C++ decoders release the GIL. ``take()`` returns the next item (waiting for it if
    needed) and immediately starts producing the one after."""

    def __init__(self, fn, *args, **kw):
        from concurrent.futures import ThreadPoolExecutor
        self._fn, self._args, self._kw = fn, args, kw
        self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="oni-ahead")
        self._fut = self._pool.submit(fn, *args, **kw)

    def take(self):
        out = self._fut.result()
        self._fut = self._pool.submit(self._fn, *self._args, **self._kw)
        return out

    def close(self) -> None:
        self._fut.cancel()
        self._pool.shutdown(wait=True)

