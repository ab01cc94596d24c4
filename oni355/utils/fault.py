"""Fault injection and fail-fast detection for the sweep loop.

``ONI_FAULT=rank:R,sweep:S,kind:{exit,hang,nan,raise}[,attempt:A]`` makes rank R misbehave when
it reaches sweep S:

* ``exit``  -- the process dies (``os._exit(17)``), as a crashed rank would;
* ``hang``  -- the rank stops making progress (the sweep watchdog / collective timeout fires);
* ``nan``   -- the model's counts and q table are corrupted (a negative count, a NaN q entry):
  the numerical health check after the sweep raises :class:`NumericalFault`;
* ``raise`` -- :class:`InjectedFault` is raised.
* ``capture`` -- the rank's next HIP-graph capture of the sweeps fails (raised between
  capture begin and end): every rank must then fall back to eager sweeps together
  (models/gibbs.py GibbsLDA._capture_agreed).

``attempt:A`` restricts the fault to the A-th launch of a supervised run (``ONI_RESTART_COUNT``,
set by ``oni-ml --max-restarts``), so a restarted child does not fail again at the same sweep.
Tests: tests/test_resilience_cpu.py.
"""
from __future__ import annotations

import os
import sys
import time


class InjectedFault(RuntimeError):
    pass


class NumericalFault(FloatingPointError):
    """Corrupt model state detected (non-finite q / likelihood, negative counts)."""


def parse(spec: str | None) -> dict | None:
    if not spec:
        return None
    out = {}
    for part in spec.split(","):
        k, _, v = part.partition(":")
        out[k.strip()] = v.strip()
    f = {"rank": int(out.get("rank", 0)), "sweep": int(out.get("sweep", 0)), "kind": out.get("kind", "raise")}
    if "attempt" in out:
        f["attempt"] = int(out["attempt"])
    return f


def maybe_inject(sweep: int, rank: int, corrupt=None) -> None:
    """Fire the configured fault if this rank reached its sweep. ``corrupt()`` implements ``nan``."""
    f = parse(os.environ.get("ONI_FAULT"))
    if not f or f["rank"] != rank or sweep < f["sweep"]:
        return
    if "attempt" in f and int(os.environ.get("ONI_RESTART_COUNT", "0")) != f["attempt"]:
        return
    kind = f["kind"]
    if kind == "capture":
        return  # fired by capture_fails(), inside the graph capture
    if kind == "exit":
        sys.stderr.write(f"[oni355] injected fault: exit at sweep {sweep} rank {rank}\n")
        sys.stderr.flush()
        os._exit(17)
    if kind == "hang":
        time.sleep(3600)
    if kind == "nan":
        if corrupt is None:
            raise InjectedFault("kind:nan needs a model to corrupt")
        corrupt()
        return
    raise InjectedFault(f"injected fault at sweep {sweep} rank {rank}")


def capture_fails(rank: int) -> bool:
    """Should this rank's sweep-graph capture fail (``ONI_FAULT=rank:R,kind:capture``)?"""
    f = parse(os.environ.get("ONI_FAULT"))
    if not f or f["kind"] != "capture" or f["rank"] != rank:
        return False
    return "attempt" not in f or int(os.environ.get("ONI_RESTART_COUNT", "0")) == f["attempt"]


class Watchdog:
    """Fail-fast sweep watchdog: while ARMED, if no ``kick()`` arrives for
    ``timeout_s`` seconds the process dumps all thread stacks to stderr and exits with code 75, so
    the supervisor (``oni-ml --max-restarts``) restarts the job from its last checkpoint instead
    of hanging in a wedged collective.

    The sampler arms it for the duration of each ``sweep()`` call and kicks it between graph
    pairs; outside sweeping (corpus build, scoring, CSV output) it is disarmed and never fires.
    ``ONI_SWEEP_TIMEOUT_S`` enables it from the environment (see :func:`from_env`).
    """

    EXIT_CODE = 75

    def __init__(self, timeout_s: float, on_timeout=None, armed: bool = True):
        import threading

        self.timeout_s = float(timeout_s)
        self._last = time.monotonic()
        self._armed = armed
        self._stop = threading.Event()
        self._on_timeout = on_timeout or self._default_timeout
        self._t = threading.Thread(target=self._run, name="oni-watchdog", daemon=True)
        self._t.start()

    def kick(self) -> None:
        self._last = time.monotonic()

    def arm(self) -> None:
        self._last = time.monotonic()
        self._armed = True

    def disarm(self) -> None:
        self._armed = False

    def close(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        period = min(max(self.timeout_s / 10.0, 0.01), 5.0)
        while not self._stop.wait(period):
            if self._armed and time.monotonic() - self._last > self.timeout_s:
                self._on_timeout()
                return

    def _default_timeout(self) -> None:
        import faulthandler

        sys.stderr.write(f"[oni355] watchdog: no sweep progress for {self.timeout_s:.0f}s, aborting\n")
        faulthandler.dump_traceback(all_threads=True)
        sys.stderr.flush()
        os._exit(self.EXIT_CODE)

    @staticmethod
    def from_env(armed: bool = False):
        v = os.environ.get("ONI_SWEEP_TIMEOUT_S")
        return Watchdog(float(v), armed=armed) if v else None
