"""Parallel ingest (oni-ingest master_collector.py + worker.py).

Reference: a watchdog Observer publishes each new file path to a Kafka topic; N worker processes
consume partitions, decode (nfdump / tshark), ``hadoop fs -put`` and load Hive parquet partitions.

Here (single node, no Kafka/HDFS): a collector polls ``collector_path`` for files matching
``supported_files``, waits until a file's size is stable, and hands it to a thread pool; each
worker decodes with the native C++ decoders (which release the GIL) and appends the rows to the
day-partitioned columnar store, split by the UTC day of each row's timestamp. Processed files are
recorded in ``<collector_path>/.oni_ingested`` (idempotent restarts) and optionally moved away.
"""
from __future__ import annotations

import concurrent.futures as cf
import datetime as _dt
import fnmatch
import json
import os
import shutil
import threading
import time

import numpy as np

from ..store import columnar
from ..store.columnar import StringColumn

DEFAULT_PATTERNS = {"flow": ["nfcapd.*", "*.csv"], "dns": ["*.pcap", "*.pcapng"], "proxy": ["*.log"]}


def decode_file(source: str, path: str) -> dict:
    from ..io import decoders
    if source == "flow":
        if path.endswith(".csv") or path.endswith(".txt"):
            return decoders.read_flow_csv(path)[0]
        from ..io import nfcapd
        return nfcapd.read_nfcapd(path)
    if source == "dns":
        return {k: v for k, v in decoders.read_pcap_dns(path).items() if not k.startswith("_")}
    return {k: v for k, v in decoders.read_proxy_log(path).items() if not k.startswith("_")}


def _fixed_digits(col, offs: list[int]) -> np.ndarray:
    """Integer made of the ASCII digits at byte offsets ``offs`` of every string (fixed-width
    fields such as p_date "YYYY-MM-DD" / p_time "HH:MM:SS"), vectorised; short strings -> 0."""
    o, ln = col.offsets[:-1], np.diff(col.offsets)
    ok = ln > max(offs)
    v = np.zeros(len(col), np.int64)
    for k in offs:
        d = np.zeros(len(col), np.int64)
        d[ok] = col.chars[o[ok] + k].astype(np.int64) - 48
        v = v * 10 + d
    return np.where(ok, v, 0)


def _row_day_hour(source: str, cols: dict) -> tuple[np.ndarray, np.ndarray]:
    """(days since epoch, hour of day) of every row."""
    if source in ("flow", "dns"):
        t = np.asarray(cols["unix_tstamp"], np.int64)
        return (t // 86400).astype(np.int64), (t % 86400) // 3600
    y = _fixed_digits(cols["p_date"], [0, 1, 2, 3])
    m = _fixed_digits(cols["p_date"], [5, 6])
    d = _fixed_digits(cols["p_date"], [8, 9])
    ok = (y > 0) & (m >= 1) & (m <= 12) & (d >= 1)
    months = np.where(ok, (y - 1970) * 12 + (m - 1), 0).astype("datetime64[M]")
    days = (months.astype("datetime64[D]").astype(np.int64) + np.where(ok, d - 1, 0))
    return np.where(ok, days, 0), np.clip(_fixed_digits(cols["p_time"], [0, 1]), 0, 23)


def _row_days(source: str, cols: dict) -> np.ndarray:
    return _row_day_hour(source, cols)[0]


def store_rows(root: str, source: str, cols: dict, hourly: bool = True) -> dict[str, int]:
    """Append decoded rows to their day (and hour) partitions; returns {YYYYMMDD: rows}."""
    days, hrs = _row_day_hour(source, cols)
    key = days * 24 + hrs if hourly else days
    out: dict[str, int] = {}
    order = np.argsort(key, kind="stable")
    uk, first = np.unique(key[order], return_index=True)
    bounds = list(first) + [key.size]
    for j, k in enumerate(uk.tolist()):
        idx = order[bounds[j]:bounds[j + 1]]
        part = {c: (v.take(idx) if isinstance(v, StringColumn) else np.asarray(v)[idx]) for c, v in cols.items()}
        day = k // 24 if hourly else k
        date = (_dt.date(1970, 1, 1) + _dt.timedelta(days=int(day))).strftime("%Y%m%d")
        columnar.append_part(root, source, date, part, hour=int(k % 24) if hourly else None)
        out[date] = out.get(date, 0) + int(idx.size)
    return out


class Collector:
    def __init__(self, source: str, collector_path: str, data_root: str, patterns=None, workers: int = 4,
                 move_to: str | None = None, log=print):
        self.source = source
        self.path = collector_path
        self.root = data_root
        self.patterns = patterns or DEFAULT_PATTERNS[source]
        self.pool = cf.ThreadPoolExecutor(max_workers=workers)
        self.move_to = move_to
        self.log = log
        self.state_file = os.path.join(collector_path, ".oni_ingested")
        self.done = set()
        if os.path.exists(self.state_file):
            with open(self.state_file) as f:
                self.done = {ln.strip() for ln in f if ln.strip()}
        self.lock = threading.Lock()
        self.sizes: dict[str, int] = {}
        self.stats = {"files": 0, "rows": 0, "errors": 0}

    def _candidates(self) -> list[str]:
        out = []
        for name in sorted(os.listdir(self.path)):
            p = os.path.join(self.path, name)
            if name.startswith(".") or not os.path.isfile(p) or name in self.done:
                continue
            if any(fnmatch.fnmatch(name, pat) for pat in self.patterns):
                out.append(p)
        return out

    def _stable(self, p: str) -> bool:
        s = os.path.getsize(p)
        prev = self.sizes.get(p)
        self.sizes[p] = s
        return prev == s

    def _work(self, p: str) -> dict:
        t0 = time.perf_counter()
        cols = decode_file(self.source, p)  # parallel: the C++ decoders release the GIL
        with self.lock:  # part numbering is per day directory: serialise the appends
            per_day = store_rows(self.root, self.source, cols)
            name = os.path.basename(p)
            self.done.add(name)
            with open(self.state_file, "a") as f:
                f.write(name + "\n")
            self.stats["files"] += 1
            self.stats["rows"] += sum(per_day.values())
        if self.move_to:
            os.makedirs(self.move_to, exist_ok=True)
            shutil.move(p, os.path.join(self.move_to, os.path.basename(p)))
        rec = {"file": p, "days": per_day, "seconds": time.perf_counter() - t0}
        self.log(json.dumps(rec))
        return rec

    def run_once(self, wait_stable: bool = False) -> list[dict]:
        files = [p for p in self._candidates() if (not wait_stable or self._stable(p))]
        futs = [self.pool.submit(self._work, p) for p in files]
        out = []
        for f in futs:
            try:
                out.append(f.result())
            except Exception as e:  # noqa: BLE001 - keep the collector alive, report the file
                self.stats["errors"] += 1
                self.log(json.dumps({"error": str(e)}))
        return out

    def watch(self, interval: float = 5.0, stop: threading.Event | None = None) -> None:
        stop = stop or threading.Event()
        while not stop.is_set():
            self.run_once(wait_stable=True)
            stop.wait(interval)
