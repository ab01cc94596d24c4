#!/usr/bin/env python3
"""Count the instructions of a kernel's hottest loop in an amdgcn assembly file (hipcc -S).

Usage: python tools/isa_loop.py <file.s> <kernel-symbol-substring>

Finds the kernel's body, splits it into basic blocks, takes every block inside the largest
back-edge range (the token loop of a sampler) and prints instruction counts by class (VALU,
SALU, VMEM, LDS, branches, waits) plus the top mnemonics. Used to check instruction-count
claims against the disassembly instead of the source (docs/performance.md).
"""
import collections
import re
import sys


def kernel_lines(path, sym):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if start is None and l.startswith("_Z") and sym in l.split(":")[0] and l.rstrip().endswith(sym.split()[-1]) is not None and ":" in l:
            if sym in l.split(":")[0]:
                start = i
                continue
        if start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i + 1]
    raise SystemExit(f"kernel {sym} not found")


def classify(m):
    if m.startswith("v_") and not m.startswith("v_readfirstlane"):
        return "VALU"
    if m.startswith("s_waitcnt"):
        return "WAIT"
    if m.startswith("s_cbranch") or m.startswith("s_branch"):
        return "BRANCH"
    if m.startswith("s_"):
        return "SALU"
    if m.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if m.startswith("ds_"):
        return "LDS"
    return "OTHER"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, sym)
    labels = {}
    insts = []  # (index, label-or-None, mnemonic, text)
    for l in body:
        s = l.split(";")[0].strip()
        if not s or s.startswith((";", ".")) and not s.startswith(".LBB"):
            continue
        if s.startswith(".LBB") and s.endswith(":"):
            labels[s[:-1]] = len(insts)
            continue
        m = s.split()[0]
        insts.append((m, s))
    # back edges: branch to a label defined earlier
    best = None
    for i, (m, s) in enumerate(insts):
        if m.startswith(("s_cbranch", "s_branch")):
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                span = (labels[tgt], i)
                if best is None or span[1] - span[0] > best[1] - best[0]:
                    best = span
    if best is None:
        raise SystemExit("no loop found")
    loop = insts[best[0]: best[1] + 1]
    cls = collections.Counter(classify(m) for m, _ in loop)
    mn = collections.Counter(m for m, _ in loop if classify(m) == "VALU")
    print(f"kernel body {len(insts)} instructions; largest loop {len(loop)} instructions")
    for k, v in sorted(cls.items(), key=lambda x: -x[1]):
        print(f"  {k:7s} {v}")
    print("  top VALU mnemonics:")
    for m, v in mn.most_common(25):
        print(f"    {m:28s} {v}")


if __name__ == "__main__":
    main()
