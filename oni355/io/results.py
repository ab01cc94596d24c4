"""ML results CSV writer/reader (``<LPATH>/<source>/<YYYYMMDD>/<source>_results.csv``).

Schema: raw columns in SURVEY.md §2.7 order + derived words + scores, ascending by score
(``oni355.schema.*_RESULT_COLUMNS``; the reference's exact order is unverifiable, §0 F1).
The reference produced it with ``hdfs dfs -getmerge`` of Spark part files ([U-M]).
"""
from __future__ import annotations

import csv
import datetime as _dt
import os

import numpy as np

from .. import schema
from ..ref import spec


def ip_str(v) -> str:
    v = int(v) & 0xFFFFFFFF
    return f"{v >> 24}.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}"


def _fmt_time(unix) -> str:
    return _dt.datetime.fromtimestamp(int(unix), tz=_dt.timezone.utc).strftime("%Y-%m-%d %H:%M:%S")


def _fmt(col: str, v) -> str:
    if col in schema.FLOW_IP_COLUMNS:
        return ip_str(v)
    if col in schema.FLOW_TIME_COLUMNS:
        return _fmt_time(v)
    if col in schema.FLOW_FLOAT_COLUMNS:
        return f"{float(v):g}"
    if isinstance(v, (float, np.floating)):
        return repr(float(v))
    return str(v)


def flow_rows(cols: dict, local_rows: np.ndarray, src_words, dst_words, src_scores, dst_scores, scores) -> list[list]:
    out = []
    for i, r in enumerate(np.asarray(local_rows, dtype=np.int64)):
        row = [_fmt(c, cols[c][r]) for c in schema.FLOW_COLUMNS]
        row += [spec.flow_word_str(int(src_words[i])), spec.flow_word_str(int(dst_words[i])),
                f"{float(src_scores[i]):.9g}", f"{float(dst_scores[i]):.9g}", f"{float(scores[i]):.9g}"]
        out.append(row)
    return out


_EVENT_IP_COLUMNS = {"ip_src", "ip_dst", "clientip", "serverip"}


def event_rows(source: str, cols: dict, local_rows, words: list[str], scores) -> list[list]:
    """DNS / proxy result rows: raw columns in schema order + word + score."""
    names = schema.raw_columns(source)
    out = []
    for i, r in enumerate(np.asarray(local_rows, dtype=np.int64)):
        row = []
        for c in names:
            v = cols.get(c)
            if v is None:
                row.append("")
            elif hasattr(v, "offsets"):
                row.append(v[int(r)])
            elif c in _EVENT_IP_COLUMNS:
                row.append(ip_str(v[r]))
            else:
                row.append(str(v[r]))
        if source == "dns" and not row[0]:
            row[0] = _fmt_time(cols["unix_tstamp"][r])
        out.append(row + [words[i], f"{float(scores[i]):.9g}"])
    return out


def render_result(source: str, cols: dict, res, row_off: int, comm=None) -> list[list]:
    """Result rows of a pipeline run (FlowResult / SingleResult) as CSV fields, ascending score.

    Each rank renders the result rows it holds (``cols`` is its shard, starting at global row
    ``row_off``); with a process group the rendered rows are gathered (collective X06's payload)
    and every rank returns the full, globally ordered list."""
    rows_local = res.rows - row_off
    if source == "flow":
        mine = (rows_local >= 0) & (rows_local < len(cols["sip"]))
        rendered = flow_rows(cols, rows_local[mine], res.src_words[mine], res.dst_words[mine],
                             res.src_scores[mine], res.dst_scores[mine], res.scores[mine])
    else:
        if source == "dns":
            from ..pipeline.dns import word_str
        else:
            from ..pipeline.proxy import word_str
        ncol = len(cols["ip_dst" if source == "dns" else "clientip"])
        mine = (rows_local >= 0) & (rows_local < ncol)
        rendered = event_rows(source, cols, rows_local[mine], [word_str(w) for w in res.words[mine]],
                              res.scores[mine])
    if comm is None or not comm.dist:
        return rendered
    import torch.distributed as dist
    gids = res.rows[mine].tolist()
    allp = [None] * comm.world
    dist.all_gather_object(allp, (gids, rendered), group=comm.group)
    by_gid = {g: r for gl, rl in allp for g, r in zip(gl, rl)}
    return [by_gid[int(g)] for g in res.rows.tolist()]


def write_csv(path: str, header: list[str], rows: list[list], with_header: bool = True) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w", newline="") as f:
        w = csv.writer(f)
        if with_header:
            w.writerow(header)
        w.writerows(rows)
    os.replace(tmp, path)
    return path


def read_csv(path: str) -> tuple[list[str], list[list[str]]]:
    with open(path, newline="") as f:
        r = csv.reader(f)
        header = next(r)
        return header, [row for row in r]


def results_path(lpath: str, source: str, date: str) -> str:
    return os.path.join(lpath, source, date, f"{source}_results.csv")


def scores_path(lpath: str, source: str, date: str | None = None) -> str:
    """Feedback file the next ML run reads (reference: ${LPATH}/${DSOURCE}_scores.csv)."""
    if date:
        return os.path.join(lpath, source, date, f"{source}_scores.csv")
    return os.path.join(lpath, f"{source}_scores.csv")
