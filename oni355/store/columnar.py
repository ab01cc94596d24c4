"""Day/hour-partitioned columnar store (replaces the reference's HDFS + Hive/Parquet tables partitioned
by y/m/d/h).

Layout::

    <root>/<source>/<YYYYMMDD>/_schema.json        {"rows": N, "columns": {name: kind}, ...}
    <root>/<source>/<YYYYMMDD>/<col>.npy           numeric column (np.save, no pickle)
    <root>/<source>/<YYYYMMDD>/<col>.off.npy       string column: int64 offsets [N+1]
    <root>/<source>/<YYYYMMDD>/<col>.chars.bin     string column: UTF-8 bytes
    <root>/<source>/<YYYYMMDD>/hHH/part-XXXXX/      hour partitions written by ingest (y/m/d/h)

Numeric columns are memory-mapped on read, so a rank of a data-parallel job touches only its own
row range; strings stay as offsets+bytes (the GPU string kernels' native layout). Appends
(ingest) go to numbered parts ``part-XXXXX/`` that readers concatenate.
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np


class StringColumn:
    """Offsets + bytes view of N strings."""

    def __init__(self, offsets: np.ndarray, chars: np.ndarray):
        self.offsets = np.asarray(offsets, dtype=np.int64)
        self.chars = np.asarray(chars, dtype=np.uint8)

    @classmethod
    def from_list(cls, items) -> "StringColumn":
        enc = [s.encode("utf-8") if isinstance(s, str) else bytes(s) for s in items]
        off = np.zeros(len(enc) + 1, dtype=np.int64)
        if enc:
            off[1:] = np.cumsum([len(e) for e in enc])
        return cls(off, np.frombuffer(b"".join(enc), dtype=np.uint8).copy())

    def __len__(self) -> int:
        return self.offsets.size - 1

    def __getitem__(self, i):
        if isinstance(i, (int, np.integer)):
            return bytes(self.chars[self.offsets[i]:self.offsets[i + 1]]).decode("utf-8", "replace")
        idx = np.arange(len(self))[i] if isinstance(i, slice) else np.asarray(i)
        return StringColumn.from_list([self[int(j)] for j in idx])

    def take(self, idx) -> "StringColumn":
        """Gather rows ``idx`` (vectorised: one fancy-index over the bytes, no per-row Python)."""
        idx = np.asarray(idx, dtype=np.int64)
        lo, hi = self.offsets[idx], self.offsets[idx + 1]
        ln = hi - lo
        off = np.zeros(idx.size + 1, dtype=np.int64)
        np.cumsum(ln, out=off[1:])
        src = np.repeat(lo - off[:-1], ln) + np.arange(int(off[-1]), dtype=np.int64)
        return StringColumn(off, self.chars[src])

    def slice(self, lo: int, hi: int) -> "StringColumn":
        o = self.offsets[lo:hi + 1]
        return StringColumn(o - o[0], self.chars[o[0]:o[-1]])

    def to_list(self) -> list[str]:
        return [self[i] for i in range(len(self))]

    @staticmethod
    def join_rows(pieces: list) -> "StringColumn":
        """Row-wise concatenation without per-row Python: ``pieces`` are (StringColumn | bytes,
        include-mask or None) pairs; row i of the result is the concatenation of every piece whose
        mask is true at i (a bytes piece is the same literal on every row)."""
        n = None
        for c, m in pieces:
            if isinstance(c, StringColumn):
                n = len(c)
            elif m is not None:
                n = len(m)
            if n is not None:
                break
        n = 0 if n is None else n
        lens = []
        for c, m in pieces:
            ln = (np.diff(c.offsets) if isinstance(c, StringColumn) else np.full(n, len(c), np.int64))
            lens.append(ln if m is None else np.where(m, ln, 0))
        tot = np.sum(lens, axis=0) if lens else np.zeros(n, np.int64)
        off = np.zeros(n + 1, np.int64)
        np.cumsum(tot, out=off[1:])
        out = np.empty(int(off[-1]), np.uint8)
        pos = off[:-1].copy()
        for (c, m), ln in zip(pieces, lens):
            k = int(ln.sum())
            if k:
                dst = np.repeat(pos, ln) + (np.arange(k, dtype=np.int64) - np.repeat(np.cumsum(ln) - ln, ln))
                if isinstance(c, StringColumn):
                    src = np.repeat(c.offsets[:-1], ln) + (dst - np.repeat(pos, ln))
                    out[dst] = c.chars[src]
                else:
                    lit = np.frombuffer(c, np.uint8)
                    out[dst] = lit[dst - np.repeat(pos, ln)]
            pos += ln
        return StringColumn(off, out)

    @staticmethod
    def from_fixed(a: np.ndarray) -> "StringColumn":
        """[n, w] uint8 rows (fixed-width strings) → StringColumn."""
        a = np.ascontiguousarray(a, dtype=np.uint8)
        n, w = a.shape
        return StringColumn(np.arange(n + 1, dtype=np.int64) * w, a.reshape(-1))

    @staticmethod
    def concat(parts: list["StringColumn"]) -> "StringColumn":
        if not parts:
            return StringColumn(np.zeros(1, np.int64), np.zeros(0, np.uint8))
        offs, base = [np.zeros(1, np.int64)], 0
        for p in parts:
            offs.append(p.offsets[1:] + base)
            base += int(p.offsets[-1])
        return StringColumn(np.concatenate(offs), np.concatenate([p.chars for p in parts]))


def day_dir(root: str, source: str, date: str) -> str:
    return os.path.join(root, source, date)


def _write_part(d: str, cols: dict) -> int:
    os.makedirs(d, exist_ok=True)
    n = None
    kinds = {}
    for name, v in cols.items():
        if isinstance(v, StringColumn) or (isinstance(v, (list, tuple)) and (not v or isinstance(v[0], str))):
            sc = v if isinstance(v, StringColumn) else StringColumn.from_list(v)
            np.save(os.path.join(d, f"{name}.off.npy"), sc.offsets, allow_pickle=False)
            sc.chars.tofile(os.path.join(d, f"{name}.chars.bin"))
            kinds[name] = "string"
            m = len(sc)
        else:
            a = np.asarray(v)
            np.save(os.path.join(d, f"{name}.npy"), a, allow_pickle=False)
            kinds[name] = str(a.dtype)
            m = a.shape[0]
        if n is not None and m != n:
            raise ValueError(f"column {name} has {m} rows, expected {n}")
        n = m
    meta = {"rows": int(n or 0), "columns": kinds}
    with open(os.path.join(d, "_schema.json.tmp"), "w") as f:
        json.dump(meta, f)
    os.replace(os.path.join(d, "_schema.json.tmp"), os.path.join(d, "_schema.json"))
    return int(n or 0)


def write_day(root: str, source: str, date: str, cols: dict) -> str:
    """Replace the day's table with ``cols`` (idempotent rerun, like ``hdfs dfs -rm`` + load);
    a whole-day write is complete on return (``_SUCCESS``)."""
    d = day_dir(root, source, date)
    if os.path.isdir(d):
        for p in glob.glob(os.path.join(d, "**", "*"), recursive=True):
            if os.path.isfile(p):
                os.remove(p)
    _write_part(d, cols)
    mark_complete(root, source, date)
    return d


def mark_complete(root: str, source: str, date: str) -> None:
    """Declare a day's ingest finished (Hadoop's ``_SUCCESS`` marker): ``oni-ml --follow`` only
    trains days that are complete."""
    d = day_dir(root, source, date)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "_SUCCESS"), "w"):
        pass


def days(root: str, source: str, complete_only: bool = True) -> list[str]:
    """Stored days of a source (YYYYMMDD, ascending); ``complete_only``: only days with a
    ``_SUCCESS`` marker."""
    base = os.path.join(root, source)
    out = []
    for d in sorted(glob.glob(os.path.join(base, "[0-9]" * 8))):
        if os.path.isdir(d) and (not complete_only or os.path.exists(os.path.join(d, "_SUCCESS"))):
            out.append(os.path.basename(d))
    return out


def hour_dir(root: str, source: str, date: str, hour: int) -> str:
    return os.path.join(day_dir(root, source, date), f"h{int(hour):02d}")


def append_part(root: str, source: str, date: str, cols: dict, hour: int | None = None) -> str:
    """Append one ingested file's rows as a new part (used by the ingest workers). With ``hour``
    the part goes to the day's hour partition ``hHH/`` (the reference's y/m/d/h Hive
    partitioning), so hourly OA drill-downs read only that hour."""
    d = day_dir(root, source, date) if hour is None else hour_dir(root, source, date, hour)
    os.makedirs(d, exist_ok=True)
    existing = sorted(p for p in glob.glob(os.path.join(d, "part-*")) if not p.endswith(".tmp"))
    nxt = 0 if not existing else int(os.path.basename(existing[-1])[5:]) + 1
    p = os.path.join(d, f"part-{nxt:05d}")
    _write_part(p + ".tmp", cols)
    os.replace(p + ".tmp", p)
    return p


def hours(root: str, source: str, date: str) -> list[int]:
    """Hour partitions present for a day."""
    d = day_dir(root, source, date)
    return sorted(int(os.path.basename(h)[1:]) for h in glob.glob(os.path.join(d, "h[0-9][0-9]")) if os.path.isdir(h))


def _parts(d: str, hour_list=None) -> list[str]:
    """Day-level table + day-level parts (unless only some hours are asked for), then the parts of
    every hour partition in hour order."""
    parts = []
    if hour_list is None:
        if os.path.exists(os.path.join(d, "_schema.json")):
            parts.append(d)
        parts += sorted(p for p in glob.glob(os.path.join(d, "part-*")) if not p.endswith(".tmp"))
    for h in sorted(glob.glob(os.path.join(d, "h[0-9][0-9]"))):
        if hour_list is not None and int(os.path.basename(h)[1:]) not in hour_list:
            continue
        parts += sorted(p for p in glob.glob(os.path.join(h, "part-*")) if not p.endswith(".tmp"))
    return parts


def rows(root: str, source: str, date: str, hours: list[int] | None = None) -> int:
    total = 0
    for p in _parts(day_dir(root, source, date), hours):
        with open(os.path.join(p, "_schema.json")) as f:
            total += json.load(f)["rows"]
    return total


def read_day(root: str, source: str, date: str, columns=None, row_range: tuple[int, int] | None = None,
             hours: list[int] | None = None, mmap: bool = False) -> dict:
    """Columns of a stored day (all partitions, or only the hour partitions in ``hours``);
    ``row_range`` selects global rows [lo, hi) of that view (a data-parallel rank's shard).
    ``mmap``: a column held by one partition is returned as a read-only memory map of the file
    (no copy: the multi-day loader reads only the device columns in full and renders a few
    thousand result rows from the rest); columns spread over partitions are concatenated."""
    d = day_dir(root, source, date)
    parts = _parts(d, hours)
    if not parts:
        raise FileNotFoundError(f"no {source} data for {date} under {root}")
    out: dict[str, list] = {}
    base = 0
    lo, hi = row_range if row_range else (0, None)
    for p in parts:
        with open(os.path.join(p, "_schema.json")) as f:
            meta = json.load(f)
        n = meta["rows"]
        plo, phi_ = max(lo - base, 0), n if hi is None else min(hi - base, n)
        base += n
        if phi_ <= plo:
            continue
        for name, kind in meta["columns"].items():
            if columns is not None and name not in columns:
                continue
            if kind == "string":
                off = np.load(os.path.join(p, f"{name}.off.npy"), mmap_mode="r" if mmap else None, allow_pickle=False)
                cpath = os.path.join(p, f"{name}.chars.bin")
                if mmap and os.path.getsize(cpath):
                    chars = np.memmap(cpath, dtype=np.uint8, mode="r")
                else:
                    chars = np.fromfile(cpath, dtype=np.uint8)
                out.setdefault(name, []).append(StringColumn(off, chars).slice(plo, phi_))
            else:
                a = np.load(os.path.join(p, f"{name}.npy"), mmap_mode="r", allow_pickle=False)
                out.setdefault(name, []).append(a[plo:phi_] if mmap else np.array(a[plo:phi_]))
    res = {}
    for k, v in out.items():
        if len(v) == 1:
            res[k] = v[0]  # one partition: no concatenation copy (a memory map with ``mmap``)
        else:
            res[k] = StringColumn.concat(v) if isinstance(v[0], StringColumn) else np.concatenate(v)
    return res
