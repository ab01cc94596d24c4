"""ctypes binding of ``oni355/_lib/liboni_native.so`` (C++ host runtime: decoders, VEM LDA)."""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(_HERE), "_lib")
NATIVE_LIB_PATH = os.path.join(LIB_DIR, "liboni_native.so")
BIN_DIR = os.path.join(LIB_DIR, "bin")

_lock = threading.Lock()
_lib = None
_SIGS: dict[str, tuple[list, object]] = {"oni_native_version": ([], C.c_int)}


def register(name: str, argtypes: list, restype=C.c_int) -> None:
    _SIGS[name] = (argtypes, restype)
    if _lib is not None and hasattr(_lib, name):
        fn = getattr(_lib, name)
        fn.argtypes, fn.restype = argtypes, restype


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(NATIVE_LIB_PATH):
                raise RuntimeError(f"{NATIVE_LIB_PATH} missing; run `python tools/build.py`")
            h = C.CDLL(NATIVE_LIB_PATH)
            for name, (args, res) in _SIGS.items():
                if hasattr(h, name):
                    fn = getattr(h, name)
                    fn.argtypes, fn.restype = args, res
            from ..utils import provenance
            h.oni_native_src_hash.restype = C.c_char_p
            h.oni_native_src_hash.argtypes = []
            provenance.check("native", h.oni_native_src_hash().decode(), NATIVE_LIB_PATH)
            _lib = h
    return _lib


def binary(name: str) -> str:
    p = os.path.join(BIN_DIR, name)
    if not os.path.exists(p):
        raise RuntimeError(f"{p} missing; run `python tools/build.py`")
    return p
