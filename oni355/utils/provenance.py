"""Build provenance: a content hash of the native sources, compiled into the libraries.

``tools/build.py`` embeds :func:`tree_hash` of the sources each library is built from
(``oni_hip_src_hash()`` in liboni_hip.so, ``oni_native_src_hash()`` in liboni_native.so), and
rebuilds objects by source *content*, not mtime. When the package loads a library from a tree that
still carries ``csrc/`` (this repository, and every gpurun snapshot of it), it compares the
embedded hash with the tree's: a library built from other sources is refused (``ONI_ALLOW_STALE=1``
downgrades that to a warning), so a GPU test run proves which sources its kernels came from.
"""
from __future__ import annotations

import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")

SOURCES = {
    "hip": ["kernels/*.hip", "kernels/*.h"],
    "native": ["native/*.cpp", "native/*.h", "io/*.cpp", "io/*.h", "lda_cpu/*.cpp", "lda_cpu/*.h"],
}


def source_files(kind: str) -> list[str]:
    out: list[str] = []
    for pat in SOURCES[kind]:
        out += glob.glob(os.path.join(CSRC, pat))
    return sorted(set(out))


def tree_hash(kind: str) -> str | None:
    """sha256 (first 16 hex digits) over the relative paths + contents of ``kind``'s sources;
    None when the tree carries no sources (an installed package)."""
    files = source_files(kind)
    if not files:
        return None
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, CSRC).encode())
        h.update(b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def check(kind: str, embedded: str | None, lib_path: str) -> None:
    want = tree_hash(kind)
    if want is None or embedded is None:
        return
    if embedded != want:
        msg = (f"{lib_path} was built from {kind} sources {embedded}, this tree has {want}: "
               f"rebuild with `python tools/build.py`")
        if os.environ.get("ONI_ALLOW_STALE", "0") == "1":
            import warnings
            warnings.warn(msg)
        else:
            raise RuntimeError(msg)
