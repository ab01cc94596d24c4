"""ctypes binding order (regression): a launcher module imported AFTER the HIP library was first
loaded must still get its C signature bound. Unbound ctypes functions pass Python ints as 32-bit
C ints, silently truncating 64-bit device pointers (a combined flow → DNS run hung on exactly
this: the DNS string kernels were imported lazily after the flow kernels had loaded the library).
The library loads without a GPU, so this runs on CPU."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PROBE = r"""
import ctypes as C
from oni355.ops import _lib
h = _lib.lib()                      # first load: only the core signatures are known
from oni355.ops import strings      # noqa: F401  registers its launchers late
missing = [n for n in _lib._OPTIONAL_SIGS if hasattr(h, n) and getattr(h, n).argtypes is None]
missing += [n for n in _lib._SIGS if getattr(h, n).argtypes is None]
assert not missing, missing
assert h.oni_domain_features.argtypes[0] is C.c_void_p and len(h.oni_domain_features.argtypes) == 20
print("bound", len(_lib._SIGS) + len(_lib._OPTIONAL_SIGS))
"""


def test_late_registered_launchers_are_bound():
    from oni355.ops import _lib
    if not os.path.exists(_lib.HIP_LIB_PATH):
        pytest.skip("liboni_hip.so not built")
    r = subprocess.run([sys.executable, "-c", _PROBE], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env={**os.environ, "PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "bound" in r.stdout


def test_libraries_embed_the_hash_of_this_trees_sources():
    """Build provenance: each library reports the content hash of the sources it was built from,
    which must equal this tree's (the loader refuses a stale build; a GPU run of this test
    therefore proves its kernels came from the committed sources)."""
    from oni355.ops import _lib, native
    from oni355.utils import provenance
    if not os.path.exists(_lib.HIP_LIB_PATH):
        pytest.skip("liboni_hip.so not built")
    assert _lib.lib().oni_hip_src_hash().decode() == provenance.tree_hash("hip")
    assert native.lib().oni_native_src_hash().decode() == provenance.tree_hash("native")
    r = subprocess.run([sys.executable, "-c", "from oni355.utils import provenance as p; "
                        "p.check('hip', 'deadbeefdeadbeef', 'x.so')"], cwd=ROOT, capture_output=True, text=True,
                       env={**os.environ, "PYTHONPATH": ROOT})
    assert r.returncode != 0 and "rebuild" in r.stderr
