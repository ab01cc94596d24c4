"""Day after day: the product path gets the bench's overlap (``oni-ml`` with a date range or
``--follow``, ``bench.py --from-store``).

The reference ran ingest → load → transform → ML continuously, one ``ml_ops.sh`` batch per day
([R README.md:35-38]). One process here walks a sequence of days with every host
stage overlapped with the GPU:

    day k+1: read from the columnar store + IPv6 keying + pin           (host thread)
    day k+1: device columns upload on the Prefetcher's copy stream     (copy engine)
    day k  : featurize → corpus → Gibbs → score → top-N                 (GPU)
    day k-1: result rows formatted, then gathered + written            (host thread, main thread)

The loader thread's only collective (the IPv6 dictionary of a DP day) runs on a gloo group of its
own (:meth:`oni355.parallel.comm.Comm.host_side`), so it never interleaves with the device
collectives the main thread issues.
"""
from __future__ import annotations

import os
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import torch

from ..io import results as rio
from ..io import staging
from ..store import columnar


@dataclass
class HostDay:
    date: str
    cols: dict           # this rank's rows (host), IPv6-keyed for flows
    row_off: int         # global row id of its first row
    n_total: int         # rows of the whole day
    feedback: dict | None
    pinned: dict | None  # page-locked device columns (GPU runs)
    load_s: float        # read + key + pin seconds (on the loader thread)
    extra: dict = field(default_factory=dict)


def load_host_day(source: str, root: str, date: str, rank: int, world: int, device, host_comm=None,
                  feedback_path: str | None = None, cols: dict | None = None,
                  slots: staging.PinnedSlots | None = None) -> HostDay:
    """Read this rank's share of a stored day (``cols``: already in memory instead), key IPv6
    documents (flows) and pin the device columns. Runs on the loader thread.

    The day is memory-mapped (columnar.read_day(mmap=True)): only the device columns are read in
    full, by the parallel copy into reusable pinned ``slots``; the other columns are touched only
    for the few thousand result rows rendered at the end of the day."""
    t0 = time.perf_counter()
    if cols is None:
        n = columnar.rows(root, source, date)
        per = n // world
        lo = rank * per
        hi = n if rank == world - 1 else lo + per
        cols = columnar.read_day(root, source, date, row_range=(lo, hi), mmap=True)
    else:
        n = len(cols["sip" if source == "flow" else ("ip_dst" if source == "dns" else "clientip")])
        lo = 0
    fb = None
    if feedback_path and os.path.exists(feedback_path):
        from ..oa import feedback as fbm
        fb = fbm.load_feedback(feedback_path, source)
    pinned, slot = None, None
    dev = torch.device(device)
    if source == "flow":
        from .flow import DEVICE_COLS, with_ipv6_keys
        cols, fb = with_ipv6_keys(cols, host_comm, (fb,)) if fb else (with_ipv6_keys(cols, host_comm), None)
        if dev.type == "cuda":
            if slots is not None:
                slot, pinned = slots.fill({k: cols[k] for k in DEVICE_COLS}, DEVICE_COLS)
            else:
                pinned = staging.Prefetcher.pin(cols, DEVICE_COLS)
    elif dev.type == "cuda":
        if source == "dns":
            from .dns import host_arrays
        else:
            from .proxy import host_arrays
        if slots is not None:
            slot, pinned = slots.fill(host_arrays(cols))
        else:
            pinned = staging.Prefetcher.pin_arrays(host_arrays(cols))
    return HostDay(date, cols, lo, n, fb, pinned, time.perf_counter() - t0, {"slot": slot})


class DayPipeline:
    """Overlap of host loading (thread), the H2D upload (copy stream) and the day being computed.

    ``load(date) -> HostDay`` runs on a worker thread. :meth:`take` returns the next day's
    HostDay with its device columns (None on the CPU), having queued the upload of the day after
    and the load of the one after that."""

    def __init__(self, load, device, slots: staging.PinnedSlots | None = None):
        self.load = load
        self.device = torch.device(device)
        self.pf = staging.Prefetcher(self.device) if self.device.type == "cuda" else None
        self.slots = slots
        self._pool = ThreadPoolExecutor(1, thread_name_prefix="oni-dayload")
        self._dates: list[str] = []
        self._cur: HostDay | None = None  # uploaded (or uploading) day
        self._fut = None                  # load of the day after it
        self.wait_s = 0.0                 # main-thread time spent waiting for the loader

    def extend(self, dates) -> None:
        """Queue more days (``--follow`` discovers them while it runs)."""
        self._dates.extend(dates)
        if self._cur is None and self._fut is None and self._dates:
            self._fut = self._pool.submit(self.load, self._dates.pop(0))

    def _advance(self) -> HostDay | None:
        if self._fut is None:
            return None
        t0 = time.perf_counter()
        nxt = self._fut.result()
        self.wait_s += time.perf_counter() - t0
        self._fut = self._pool.submit(self.load, self._dates.pop(0)) if self._dates else None
        if self.pf is not None:
            self.pf.submit(nxt.pinned)
            if self.slots is not None and nxt.extra.get("slot") is not None:
                self.slots.mark_used(nxt.extra["slot"], self.pf.last_event())
        return nxt

    def pending(self) -> bool:
        return self._cur is not None or self._fut is not None

    def take(self):
        """(HostDay, device columns or None) of the next day, or None when no day is queued."""
        if self._cur is None:
            self._cur = self._advance()
            if self._cur is None:
                return None
        day = self._cur
        dcols = self.pf.take() if self.pf is not None else None
        # the next day's upload starts now, on the copy stream, beside this day's compute
        self._cur = self._advance()
        return day, dcols

    def close(self) -> None:
        self._pool.shutdown(wait=True)
        if self.slots is not None:
            self.slots.close()


def run_day(source: str, day: HostDay, dcols, comm, kw: dict, on_train=None):
    """One day through the pipeline of ``source`` (device columns prefetched when given)."""
    args = dict(kw, comm=comm, row_offset=day.row_off, feedback=day.feedback)
    if source == "flow":
        from .flow import run_flow
        return run_flow(day.cols, device_cols=dcols, on_train=on_train, **args)
    if source == "dns":
        from .dns import run_dns
        return run_dns(day.cols, device_cols=dcols, **args)
    from .proxy import run_proxy
    return run_proxy(day.cols, device_cols=dcols, **args)


def run_days(source: str, dates: list[str], root: str, lpath: str, comm, kw: dict, device, follow: bool = False,
             poll_s: float = 5.0, idle_exit_s: float = 60.0, max_days: int = 0, feedback_path: str | None = None,
             log=None, on_day=None) -> list[dict]:
    """Score ``dates`` (then, with ``follow``, every later complete day the store receives) with
    all host work overlapped. Writes ``<lpath>/<source>/<date>/<source>_results.csv`` +
    ``metrics.jsonl`` per day (rank 0). Returns each day's metrics record."""
    from .. import schema
    from ..utils.obs import MetricsLog
    rank, world = comm.rank, comm.world
    host = comm.host_side() if comm.dist else None
    log = log or (lambda m: None)

    slots = staging.PinnedSlots() if torch.device(device).type == "cuda" else None

    def load(date):
        return load_host_day(source, root, date, rank, world, device, host, feedback_path, slots=slots)

    header = schema.result_columns(source)
    records: list[dict] = []

    def write(rendered, date):
        if rank == 0:
            out = rio.write_rendered(rio.results_path(lpath, source, date), header, rendered)
            log(f"{source} {date}: {len(rendered)} rows -> {out}")

    pipe = DayPipeline(load, device, slots)
    results = rio.ResultPipe(source, comm, write=write)
    done: set[str] = set()
    last = max(dates) if dates else None
    pipe.extend(list(dates))
    idle_since = time.perf_counter()
    try:
        while True:
            got = pipe.take() if pipe.pending() else None
            if got is None:
                if not follow or (max_days and len(records) >= max_days):
                    break
                # rank 0 alone decides both the new days and the idle exit (from its own clock) and
                # shares them: a rank leaving on its local clock while the others block in the next
                # broadcast would hang the group
                new, stop = _next_days(root, source, last, comm,
                                       idle=time.perf_counter() - idle_since > idle_exit_s)
                if new:
                    last = new[-1]
                    pipe.extend(new)
                    idle_since = time.perf_counter()
                    continue
                if stop:
                    break
                time.sleep(poll_s)
                continue
            day, dcols = got
            t0 = time.perf_counter()
            wait_total, pipe_wait0 = pipe.wait_s, getattr(pipe, "_wait_reported", 0.0)
            pipe._wait_reported = wait_total
            res = run_day(source, day, dcols, comm, kw)
            results.submit(day.cols, res, day.row_off, tag=day.date)
            rec = {"event": "oni-ml-day", "source": source, "date": day.date, "events": day.n_total, "ranks": world,
                   "load_s": round(day.load_s, 4), "day_s": round(time.perf_counter() - t0, 4),
                   "loader_wait_s": round(wait_total - pipe_wait0, 4), **{k: v for k, v in res.timings.items()},
                   **{k: v for k, v in res.stats.items() if isinstance(v, (int, float, str)) or v is None}}
            if dcols is not None and pipe.pf is not None:
                rec["h2d_copy_dev_s"] = (pipe.pf.copy_ms() or 0.0) / 1e3
            records.append(rec)
            if rank == 0:
                d = os.path.dirname(rio.results_path(lpath, source, day.date))
                os.makedirs(d, exist_ok=True)
                MetricsLog(os.path.join(d, "metrics.jsonl")).write(rec)
            if on_day is not None:
                on_day(day, res)
            done.add(day.date)
            if max_days and len(records) >= max_days:
                break
    finally:
        results.close()
        pipe.close()
    return records


def _next_days(root: str, source: str, after: str | None, comm, idle: bool = False) -> tuple[list[str], bool]:
    """(complete stored days after ``after``, stop) -- both decided by rank 0 and shared, so every
    rank walks the same days in the same order and leaves the ``--follow`` loop in the same pass.
    ``stop`` is rank 0's ``idle`` when it found no new day."""
    days = [d for d in columnar.days(root, source) if after is None or d > after] if comm.rank == 0 else []
    stop = bool(idle) and not days
    if comm.dist:
        import torch.distributed as dist
        box = [(days, stop)]
        dist.broadcast_object_list(box, src=0, group=comm.host_side().group)
        days, stop = box[0]
    return days, stop


def parse_dates(spec: str) -> list[str]:
    """``YYYYMMDD``, ``YYYYMMDD-YYYYMMDD`` (inclusive, calendar days) or a comma list of either."""
    import datetime as dt
    out: list[str] = []
    for part in spec.split(","):
        part = part.strip()
        if "-" in part:
            a, b = (dt.datetime.strptime(x, "%Y%m%d").date() for x in part.split("-", 1))
            if b < a:
                raise ValueError(f"empty date range {part}")
            out += [(a + dt.timedelta(days=i)).strftime("%Y%m%d") for i in range((b - a).days + 1)]
        else:
            dt.datetime.strptime(part, "%Y%m%d")
            out.append(part)
    return out
