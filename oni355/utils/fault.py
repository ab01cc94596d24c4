"""Fault injection for the sweep loop.

``ONI_FAULT=rank:R,sweep:S,kind:{exit,hang,nan,raise}`` makes rank R misbehave when it reaches
sweep S. Used by tests/test_fault.py to exercise the fail-fast + resume-from-checkpoint path.
"""
from __future__ import annotations

import os
import sys
import time


class InjectedFault(RuntimeError):
    pass


def parse(spec: str | None) -> dict | None:
    if not spec:
        return None
    out = {}
    for part in spec.split(","):
        k, _, v = part.partition(":")
        out[k.strip()] = v.strip()
    return {"rank": int(out.get("rank", 0)), "sweep": int(out.get("sweep", 0)), "kind": out.get("kind", "raise")}


def maybe_inject(sweep: int, rank: int) -> None:
    f = parse(os.environ.get("ONI_FAULT"))
    if not f or f["rank"] != rank or sweep < f["sweep"]:
        return
    kind = f["kind"]
    if kind == "exit":
        sys.stderr.write(f"[oni355] injected fault: exit at sweep {sweep} rank {rank}\n")
        os._exit(17)
    if kind == "hang":
        time.sleep(3600)
    raise InjectedFault(f"injected fault at sweep {sweep} rank {rank}")
