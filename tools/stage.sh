#!/bin/bash
# Freeze the current tree (sources + built libraries) into gpurun_stage/ for `STAGE=1 bash
# tools/gpu.sh ...`: a gpurun call snapshots the tree only when it gets a box, which can be many
# minutes after it was started; the stage keeps the call on the tree it was started for.
set -e
cd "$(dirname "$0")/.."
# refuse to freeze a library built from other sources than the tree's (the box would refuse it)
python3 - <<'PY'
import ctypes, sys
sys.path.insert(0, ".")
from oni355.utils import provenance
h = ctypes.CDLL("oni355/_lib/liboni_hip.so")
h.oni_hip_src_hash.restype = ctypes.c_char_p
got, want = h.oni_hip_src_hash().decode(), provenance.tree_hash("hip")
if got != want:
    sys.exit(f"stage: liboni_hip.so built from {got}, tree has {want}: run python tools/build.py")
PY
rm -rf gpurun_stage
mkdir -p gpurun_stage
tar --exclude=./.git --exclude=./gpurun_out --exclude=./gpurun_stage --exclude=./profiles \
  --exclude='__pycache__' --exclude=./build --exclude='*_asan*' --exclude='*.log' --exclude=./gpurun_out -cf - . | tar -xf - -C gpurun_stage
echo "staged $(du -sh gpurun_stage | cut -f1)"
