"""ctypes binding of ``oni355/_lib/liboni_hip.so`` (the hand-written gfx950 kernels).

The library exposes a plain C ABI; every launcher takes raw device pointers plus the HIP stream
(``torch.cuda.current_stream().cuda_stream``) so kernels are ordered with torch's own work and are
captured by ``torch.cuda.graph`` like any other launch.

There is no fallback: if the library is missing or was built for another architecture, every
device op raises. (CPU tensors go to the NumPy reference oracle explicitly, see ``oni355.ops``.)
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  -- must be loaded first: our .so resolves libamdhip64.so.7 to torch's copy

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(_HERE), "_lib")
HIP_LIB_PATH = os.path.join(LIB_DIR, "liboni_hip.so")

_lock = threading.Lock()
_lib = None

vp, i32, i64, f32, u32 = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_uint32


class OniGibbs(C.Structure):
    """Mirror of ``struct OniGibbs`` in csrc/kernels/gibbs_sampler.h (size checked at load)."""

    _fields_ = [
        ("tok_word", vp), ("tok_z", vp), ("slice_off", vp), ("slice_len", vp),
        ("chunk_doc", vp), ("chunk_pos0", vp), ("chunk_key", vp), ("chunk_multi", vp),
        ("ndk_src", vp), ("ndk_dst", vp), ("q", vp), ("qfix", vp), ("dnwk", vp), ("dnk", vp), ("sweep_ctr", vp), ("chg_mask", vp),
        ("wpos", vp), ("z_w", vp), ("zz_w", vp), ("chg_count", vp), ("exact_guard", vp), ("tok_zlag", vp),
        ("n_slices", i64), ("K", i32), ("KS", i32), ("alpha", f32), ("seed0", u32), ("seed1", u32),
        ("nk_rep", i32), ("flags", i32),
    ]


class OniMH(C.Structure):
    """Mirror of ``struct OniMH`` in csrc/kernels/gibbs_mh.hip (size checked at load)."""

    _fields_ = [
        ("g", OniGibbs), ("walias", vp), ("wsum", vp), ("wcdf", vp), ("dalias", vp), ("mh_g", vp), ("chunk_dslot", vp),
        ("chunk_len", vp), ("kalpha", f32), ("inv_alpha", f32), ("lmax", i32), ("doc_moves", i32), ("wp", i32),
    ]


_SIGS = {
    "oni_radix_hist": [vp, i64, C.c_int, C.c_int, vp, C.c_int, u32, vp, vp],
    "oni_f32_keys": [vp, i64, vp, vp],
    "oni_i64_keys": [vp, i64, vp, vp],
    "oni_bin_keys": [vp, i64, vp, C.c_int, vp, vp],
    "oni_flow_keys": [vp, vp, vp, vp, vp, i64, vp, vp, vp, vp],
    "oni_flow_wordify": [vp, vp, vp, vp, vp, i64, vp, C.c_int, C.c_int, C.c_int, vp, vp, vp],
    "oni_sell_fill": [vp, vp, vp, i64, C.c_int, vp, vp, vp, vp, vp, vp, vp],
    "oni_sell_perm_z": [vp, vp, vp, i64, C.c_int, vp, vp, vp, vp, C.c_int, vp],
    "oni_gibbs_launch": [C.POINTER(OniGibbs), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp],
    "oni_gibbs_sizeof_args": [],
    "oni_exact_guard": [vp, vp, i64, C.c_int, C.c_int, C.c_int32, vp, vp],
    "oni_gibbs_mh_launch": [C.POINTER(OniMH), C.c_int, C.c_int, vp],
    "oni_mh_sizeof_args": [],
    "oni_mh_tables": [vp, i64, C.c_int, C.c_int, vp, vp, i64, f32, vp, vp, vp, vp, vp, f32, vp, vp],
    "oni_widen_pair": [vp, vp, i64, vp, vp],
    "oni_quantile_pick": [vp, vp, C.c_int, C.c_int, C.c_int, vp, vp, vp],
    "oni_tail_grid": [],
    "oni_tail_sums": [vp, vp, vp, vp, i64, i64, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double,
                      vp, vp, vp],
    "oni_theta_rows": [vp, i64, C.c_int, C.c_int, f32, f32, vp, C.c_int, vp],
    "oni_phi_rows": [vp, vp, i64, C.c_int, C.c_int, f32, f32, vp, C.c_int, C.c_int, vp],
    "oni_gibbs_apply": [vp, vp, vp, vp, vp, vp, vp, i64, C.c_int, C.c_int, f32, f32, vp, C.c_int, C.c_int, C.c_int,
                        vp, vp, vp, i64, vp, vp, vp, C.c_int, vp, i64, C.c_int, vp],
    "oni_recount": [vp, vp, vp, i64, vp, C.c_int, C.c_int, C.c_int, vp],
    "oni_recount_stream": [vp, vp, i64, vp, C.c_int, C.c_int, C.c_int, vp],
    "oni_delta_recount": [vp, vp, vp, vp, vp, vp, vp, i64, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp],
    "oni_copy_rows": [vp, vp, vp, i64, C.c_int, vp],
    "oni_x01_pack": [vp, vp, i64, vp, i64, vp, i64, C.c_int, i64, i64, C.c_int, C.c_int, vp, vp],
    "oni_x01_unpack": [vp, vp, i64, vp, i64, vp, i64, C.c_int, i64, i64, C.c_int, C.c_int, vp, vp],
    "oni_score": [vp, vp, C.c_int, vp, vp, vp, vp, i64, f32, vp, vp, vp, vp, vp],
    "oni_select_below": [vp, i64, f32, u32, vp, vp, vp, i64, vp],
    "oni_pair_score": [vp, vp, C.c_int, vp, vp, i64, vp, vp],
    "oni_event_min": [vp, vp, vp, i64, f32, vp, vp, vp, vp, vp],
    "oni_tile_score": [vp, vp, C.c_int, vp, vp, vp, vp, i64, vp, vp],
    "oni_wdelta_recount": [vp, vp, vp, i64, vp, C.c_int, C.c_int, vp],
}
# optional symbols (added by later kernel files); bound when present
_OPTIONAL_SIGS: dict[str, list] = {}


def _bind(h: C.CDLL, name: str, argtypes: list) -> None:
    fn = getattr(h, name)
    fn.argtypes = argtypes
    fn.restype = C.c_int


def register_optional(name: str, argtypes: list) -> None:
    """Declare a launcher's C signature. Binds at once if the library is already loaded: an
    unbound ctypes function would pass 64-bit device pointers as 32-bit C ints (silently
    truncated), so a module imported after the first kernel launch must not stay unbound."""
    with _lock:
        _OPTIONAL_SIGS[name] = argtypes
        if _lib is not None and hasattr(_lib, name):
            _bind(_lib, name, argtypes)


def lib() -> C.CDLL:
    """Load (once) and return the HIP kernel library; raise loudly if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(HIP_LIB_PATH):
            raise RuntimeError(
                f"oni355 HIP kernels not built: {HIP_LIB_PATH} missing. Run `python tools/build.py`."
            )
        h = C.CDLL(HIP_LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            _bind(h, name, args)
        for name, args in _OPTIONAL_SIGS.items():
            if hasattr(h, name):
                _bind(h, name, args)
        if h.oni_mh_sizeof_args() != C.sizeof(OniMH):
            raise RuntimeError("OniMH layout mismatch between liboni_hip.so and oni355/ops/_lib.py")
        if h.oni_gibbs_sizeof_args() != C.sizeof(OniGibbs):
            raise RuntimeError("OniGibbs ABI mismatch between Python and liboni_hip.so; rebuild")
        from ..utils import provenance
        h.oni_hip_src_hash.restype = C.c_char_p
        h.oni_hip_src_hash.argtypes = []
        provenance.check("hip", h.oni_hip_src_hash().decode(), HIP_LIB_PATH)
        _lib = h
        return h


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("HIP op called with a CPU tensor")
    if not t.is_contiguous():
        raise ValueError("HIP op needs contiguous tensors")
    return t.data_ptr()
