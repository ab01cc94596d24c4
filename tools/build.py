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

Incremental by content: an object is rebuilt when the hash of its source + every header in
``csrc/`` + its compile flags differs from the one recorded next to it (``<obj>.sha``), never by
mtime. The libraries embed the content hash of the sources they were built from
(``oni_hip_src_hash()`` / ``oni_native_src_hash()``, oni355/utils/provenance.py), which the package
checks when it loads them.
Usage: ``python tools/build.py [--jobs N] [--only hip|native] [--sanitize] [-v]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
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


sys.path.insert(0, ROOT)
from oni355.utils import provenance  # noqa: E402


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)):
        h.update(p.encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _obj_key(src: str, cmd: list[str], hdr: str) -> str:
    h = hashlib.sha256()
    with open(src, "rb") as f:
        h.update(f.read())
    h.update(hdr.encode())
    h.update("\0".join(cmd).encode())
    return h.hexdigest()


def _stale(obj: str, key: str) -> bool:
    sha = obj + ".sha"
    if not (os.path.exists(obj) and os.path.exists(sha)):
        return True
    with open(sha) as f:
        return f.read().strip() != key


def _mark(jobs: list) -> None:
    for _, o, key in jobs:
        with open(o + ".sha", "w") as f:
            f.write(key)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ... ({r.returncode})")
    if verbose and r.stderr.strip():
        sys.stderr.write(r.stderr)


def _compile_all(jobs: list, n: int, verbose: bool) -> None:
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        futs = [ex.submit(_run, job[0], verbose) for job in jobs]
        for f in futs:
            f.result()
    _mark(jobs)


def build_hip(n_jobs: int, verbose: bool) -> str:
    os.makedirs(os.path.join(OBJ, "hip"), exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    hdr = _headers_digest()
    src_hash = provenance.tree_hash("hip")
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    objs, jobs = [], []
    for s in srcs:
        o = os.path.join(OBJ, "hip", os.path.basename(s) + ".o")
        objs.append(o)
        extra = [f'-DONI_SRC_HASH="{src_hash}"'] if os.path.basename(s) == "build_info.hip" else []
        cmd = [HIPCC, *HIP_FLAGS, *extra, "-c", s, "-o", o]
        key = _obj_key(s, cmd, hdr)
        if _stale(o, key):
            jobs.append((cmd, o, key))
    _compile_all(jobs, n_jobs, verbose)
    out = os.path.join(LIBDIR, "liboni_hip.so")
    if jobs or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + ".tmp"], verbose)
        os.replace(out + ".tmp", out)
    return out


def build_native(n_jobs: int, verbose: bool, sanitize: bool) -> list[str]:
    os.makedirs(os.path.join(OBJ, "native"), exist_ok=True)
    os.makedirs(BINDIR, exist_ok=True)
    hdr = _headers_digest()
    src_hash = provenance.tree_hash("native")
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
        extra = [f'-DONI_SRC_HASH="{src_hash}"'] if os.path.basename(s) == "version.cpp" else []
        cmd = [CXX, *flags, *extra, "-c", s, "-o", o]
        key = _obj_key(s, cmd, hdr)
        if _stale(o, key):
            jobs.append((cmd, o, key))
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
