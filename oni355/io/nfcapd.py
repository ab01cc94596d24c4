"""nfcapd (nfdump LAYOUT_VERSION_1) reader/writer -- Python side of csrc/io/nfcapd.cpp (C01)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ..ops import native
from .decoders import finish_flow_cols, ipv6_text, parse_ip_spans

vp, i64 = C.c_void_p, C.c_int64
native.register("oni_nfcapd_open", [C.c_char_p], vp)
native.register("oni_nfcapd_info", [vp, vp, vp, vp, C.c_char_p, C.c_int], C.c_int)
native.register("oni_nfcapd_fetch", [vp, vp, vp, vp], C.c_int)
native.register("oni_nfcapd_fetch_v6", [vp, vp, vp], C.c_int)
native.register("oni_nfcapd_free", [vp], None)
native.register("oni_nfcapd_write", [C.c_char_p, i64] + [vp] * 20 + [C.c_int, C.c_int], i64)
native.register("oni_lzo1x_decompress", [vp, i64, vp, i64, vp], C.c_int)
native.register("oni_lz4_decompress", [vp, i64, vp, i64, vp], C.c_int)


def read_nfcapd(path: str) -> dict:
    L = native.lib()
    h = L.oni_nfcapd_open(path.encode())
    try:
        n, blocks, skipped = C.c_int64(), C.c_int64(), C.c_int64()
        err = C.create_string_buffer(256)
        if L.oni_nfcapd_info(h, C.byref(n), C.byref(blocks), C.byref(skipped), err, 256) != 0:
            raise OSError(f"{path}: {err.value.decode()}")
        m = n.value
        a64 = np.zeros((m, 8), np.int64)
        a32 = np.zeros((m, 14), np.int32)
        rip = np.zeros(m, np.uint32)
        L.oni_nfcapd_fetch(h, a64.ctypes.data, a32.ctypes.data, rip.ctypes.data)
        is6 = np.zeros(m, np.uint8)
        a6 = np.zeros((m, 32), np.uint8)
        L.oni_nfcapd_fetch_v6(h, is6.ctypes.data, a6.ctypes.data)
    finally:
        L.oni_nfcapd_free(h)
    first_s = a64[:, 0] // 1000
    cols = {
        "treceived": first_s, "tdur": ((a64[:, 1] - a64[:, 0]) / 1000.0).astype(np.float32),
        "sport": a32[:, 0], "dport": a32[:, 1], "proto": a32[:, 2], "flag": a32[:, 3], "fwd": a32[:, 4],
        "stos": a32[:, 5], "dtos": a32[:, 6], "dir": a32[:, 7], "input": a32[:, 8], "output": a32[:, 9],
        "sas": a32[:, 10], "das": a32[:, 11], "sip": a32[:, 12].view(np.uint32), "dip": a32[:, 13].view(np.uint32),
        "ipkt": a64[:, 3], "ibyt": a64[:, 4], "opkt": a64[:, 5], "obyt": a64[:, 6], "rip": rip,
    }
    cols = {k: np.ascontiguousarray(v) for k, v in cols.items()}
    if is6.any():  # IPv6 flows: addresses as text columns (sip/dip stay 0 until the pipeline keys them)
        cols["sip6"] = ipv6_text(np.ascontiguousarray(a6[:, :16]), is6)
        cols["dip6"] = ipv6_text(np.ascontiguousarray(a6[:, 16:]), is6)
    return finish_flow_cols(cols)


def write_nfcapd(path: str, cols: dict, compression: str = "none", per_block: int = 4096) -> int:
    n = len(cols["sip"])
    t = np.asarray(cols["unix_tstamp"], np.int64) * 1000
    dur = (np.asarray(cols.get("tdur", np.zeros(n)), np.float64) * 1000).astype(np.int64)
    z32 = np.zeros(n, np.int32)
    arrs = [t, t + dur, t, np.asarray(cols["sip"], np.uint32), np.asarray(cols["dip"], np.uint32),
            np.asarray(cols["sport"], np.int32), np.asarray(cols["dport"], np.int32),
            np.asarray(cols.get("proto", z32), np.int32), np.asarray(cols.get("flag", z32), np.int32),
            np.asarray(cols["ipkt"], np.int64), np.asarray(cols["ibyt"], np.int64),
            np.asarray(cols.get("opkt", np.zeros(n)), np.int64), np.asarray(cols.get("obyt", np.zeros(n)), np.int64),
            np.asarray(cols.get("input", z32), np.int32), np.asarray(cols.get("output", z32), np.int32),
            np.asarray(cols.get("sas", z32), np.int32), np.asarray(cols.get("das", z32), np.int32),
            np.asarray(cols.get("rip", np.zeros(n)), np.uint32)]
    arrs = [np.ascontiguousarray(a) for a in arrs]
    is6, a6 = None, None
    if "sip6" in cols and "dip6" in cols:
        s6, d6 = cols["sip6"], cols["dip6"]
        _, sb, sk = parse_ip_spans(s6.chars, np.stack([s6.offsets[:-1], s6.offsets[1:]], 1))
        _, db, dk = parse_ip_spans(d6.chars, np.stack([d6.offsets[:-1], d6.offsets[1:]], 1))
        is6 = np.ascontiguousarray(((sk == 1) & (dk == 1)).astype(np.uint8))
        a6 = np.ascontiguousarray(np.concatenate([sb, db], 1))
    comp = {"none": 0, "lzo": 1, "lz4": 2, "bz2": 3}[compression]
    r = native.lib().oni_nfcapd_write(path.encode(), n, *(a.ctypes.data for a in arrs),
                                      is6.ctypes.data if is6 is not None else None,
                                      a6.ctypes.data if a6 is not None else None, comp, per_block)
    if r != n:
        raise OSError(f"nfcapd write failed: {path}")
    return r


def lzo1x_decompress(data: bytes, cap: int) -> bytes:
    src = np.frombuffer(data, np.uint8)
    out = np.zeros(cap, np.uint8)
    n = C.c_int64()
    if native.lib().oni_lzo1x_decompress(src.ctypes.data, src.size, out.ctypes.data, cap, C.byref(n)) != 0:
        raise ValueError("invalid LZO1X stream")
    return out[: n.value].tobytes()


def lz4_decompress(data: bytes, cap: int) -> bytes:
    src = np.frombuffer(data, np.uint8)
    out = np.zeros(cap, np.uint8)
    n = C.c_int64()
    if native.lib().oni_lz4_decompress(src.ctypes.data, src.size, out.ctypes.data, cap, C.byref(n)) != 0:
        raise ValueError("invalid LZ4 block")
    return out[: n.value].tobytes()
