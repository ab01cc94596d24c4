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


class Watchdog:
    """Fail-fast sweep watchdog: if no ``kick()`` arrives for ``timeout_s`` seconds
    the process dumps all thread stacks to stderr and exits with code 75, so the launcher can
    restart the job from its last checkpoint instead of hanging in a wedged collective.

    ``ONI_SWEEP_TIMEOUT_S`` enables it from the environment (see :func:`from_env`).
    """

    EXIT_CODE = 75

    def __init__(self, timeout_s: float, on_timeout=None):
        import threading

        self.timeout_s = float(timeout_s)
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._on_timeout = on_timeout or self._default_timeout
        self._t = threading.Thread(target=self._run, name="oni-watchdog", daemon=True)
        self._t.start()

    def kick(self) -> None:
        self._last = time.monotonic()

    def close(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        period = min(max(self.timeout_s / 10.0, 0.01), 5.0)
        while not self._stop.wait(period):
            if time.monotonic() - self._last > self.timeout_s:
                self._on_timeout()
                return

    def _default_timeout(self) -> None:
        import faulthandler

        sys.stderr.write(f"[oni355] watchdog: no sweep progress for {self.timeout_s:.0f}s, aborting\n")
        faulthandler.dump_traceback(all_threads=True)
        sys.stderr.flush()
        os._exit(self.EXIT_CODE)

    @staticmethod
    def from_env():
        v = os.environ.get("ONI_SWEEP_TIMEOUT_S")
        return Watchdog(float(v)) if v else None
