#!/usr/bin/env python3
"""Native build for oni355 (no JIT, no hipify, no torch headers).

Produces, in-tree (so the artefacts travel with a ``gpurun`` snapshot):

* ``oni355/_lib/liboni_hip.so``    -- every hand-written CDNA4 kernel in ``csrc/kernels/*.hip``,
  compiled by ``hipcc --offload-arch=gfx950`` only, exported through a plain C ABI (loaded with
  ctypes from :mod:`oni355.ops._lib`; launches go on torch's current HIP stream).
* ``oni355/_lib/liboni_native.so`` -- the C++ host runtime: nfdump-CSV / nfcapd / pcap-DNS /
  proxy-log decoders, the lda-c-compatible variational-EM engine, CSV formatter.
* ``oni355/_lib/bin/lda``          -- standalone ``lda est|inf`` CLI (oni-lda-c equivalent).
* ``oni355/_lib/bin/oni-nfdump``   -- standalone nfcapd → CSV decoder (oni-nfdump equivalent).

Incremental: an object is rebuilt when its source or any header in ``csrc/`` is newer.
Usage: ``python tools/build.py [--jobs N] [--only hip|native] [--sanitize] [-v]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
LIBDIR = os.path.join(ROOT, "oni355", "_lib")
BINDIR = os.path.join(LIBDIR, "bin")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
ARCH = "gfx950"

HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
    # numerics are pinned: the NumPy oracle replays the sampler bit-for-bit, so no fma contraction
    "-ffp-contract=off",
    "-mcode-object-version=5",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
    "-I", os.path.join(CSRC, "kernels"),
]
CXX_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-fopenmp", "-Wall", "-Wno-unused-function",
             "-I", os.path.join(CSRC, "native")]


def _newest_header() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _stale(src: str, obj: str, hdr_t: float) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or hdr_t > t


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ... ({r.returncode})")
    if verbose and r.stderr.strip():
        sys.stderr.write(r.stderr)


def _compile_all(jobs: list[tuple[list[str], str]], n: int, verbose: bool) -> None:
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        futs = [ex.submit(_run, cmd, verbose) for cmd, _ in jobs]
        for f in futs:
            f.result()


def build_hip(n_jobs: int, verbose: bool) -> str:
    os.makedirs(os.path.join(OBJ, "hip"), exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    hdr_t = _newest_header()
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    objs, jobs = [], []
    for s in srcs:
        o = os.path.join(OBJ, "hip", os.path.basename(s) + ".o")
        objs.append(o)
        if _stale(s, o, hdr_t):
            jobs.append(([HIPCC, *HIP_FLAGS, "-c", s, "-o", o], o))
    _compile_all(jobs, n_jobs, verbose)
    out = os.path.join(LIBDIR, "liboni_hip.so")
    if jobs or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + ".tmp"], verbose)
        os.replace(out + ".tmp", out)
    return out


def build_native(n_jobs: int, verbose: bool, sanitize: bool) -> list[str]:
    os.makedirs(os.path.join(OBJ, "native"), exist_ok=True)
    os.makedirs(BINDIR, exist_ok=True)
    hdr_t = _newest_header()
    flags = list(CXX_FLAGS)
    if sanitize:
        flags += ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-O1", "-g"]
    tag = "asan" if sanitize else "rel"
    lib_srcs = sorted(glob.glob(os.path.join(CSRC, "native", "*.cpp"))
                      + glob.glob(os.path.join(CSRC, "io", "*.cpp"))
                      + glob.glob(os.path.join(CSRC, "lda_cpu", "*.cpp")))
    mains = [s for s in lib_srcs if os.path.basename(s).startswith("main_")]
    lib_srcs = [s for s in lib_srcs if s not in mains]
    objs, jobs = [], []
    for s in lib_srcs + mains:
        o = os.path.join(OBJ, "native", f"{os.path.basename(s)}.{tag}.o")
        if s in lib_srcs:
            objs.append(o)
        if _stale(s, o, hdr_t):
            jobs.append(([CXX, *flags, "-c", s, "-o", o], o))
    _compile_all(jobs, n_jobs, verbose)
    outs = []
    suffix = "_asan" if sanitize else ""
    lib = os.path.join(LIBDIR, f"liboni_native{suffix}.so")
    if objs:
        _run([CXX, "-shared", "-fopenmp", *([f for f in flags if f.startswith("-fsanitize")]), *objs,
              "-ldl", "-o", lib + ".tmp"], verbose)
        os.replace(lib + ".tmp", lib)
        outs.append(lib)
    for m in mains:
        name = os.path.basename(m)[len("main_"):-len(".cpp")].replace("_", "-")
        o = os.path.join(OBJ, "native", f"{os.path.basename(m)}.{tag}.o")
        exe = os.path.join(BINDIR, name + suffix)
        _run([CXX, "-fopenmp", *([f for f in flags if f.startswith("-fsanitize")]), o, *objs,
              "-ldl", "-o", exe + ".tmp"], verbose)
        os.replace(exe + ".tmp", exe)
        outs.append(exe)
    return outs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--only", choices=["hip", "native"], default=None)
    ap.add_argument("--sanitize", action="store_true", help="ASan/UBSan build of the host C++ library")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    t0 = time.time()
    if a.only in (None, "native"):
        for p in build_native(a.jobs, a.verbose, a.sanitize):
            print("built", os.path.relpath(p, ROOT))
    if a.only in (None, "hip") and not a.sanitize:
        print("built", os.path.relpath(build_hip(a.jobs, a.verbose), ROOT))
    print(f"build done in {time.time() - t0:.1f}s")
    return 0


if __name__ == "__main__":
    sys.exit(main())
