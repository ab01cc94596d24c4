"""Typed configuration.

Precedence (lowest → highest): built-in defaults → ``duxbay.conf``-style KEY=VALUE file (parsed,
never sourced) → ``ONI_*`` environment variables → explicit overrides (CLI flags).

Reference keys (``/etc/duxbay.conf``, [U-M]) are accepted under their original names:
TOPIC_COUNT, DUPFACTOR, TOL, MAXRESULTS, USER_DOMAIN, LPATH, HPATH, PROCESS_COUNT, ... .
The lda-c ``settings.txt`` format is parsed by :func:`parse_lda_settings`.
"""
from __future__ import annotations

import dataclasses
import os
import re
import shlex
from dataclasses import dataclass, field


@dataclass
class OniConfig:
    # ML (oni-ml / ml_ops.sh)
    TOPIC_COUNT: int = 20
    DUPFACTOR: int = 1000
    TOL: float = 1.0
    MAXRESULTS: int = 3000
    USER_DOMAIN: str = ""
    PROCESS_COUNT: int = 1          # = GPU count (one process per GPU)
    # Gibbs sampler (our additions; lda-c settings map onto these)
    SWEEPS: int = 200
    BURNIN: int = 0
    ALPHA: float = -1.0             # <= 0: 50/K
    BETA: float | None = None  # None: models.gibbs.default_beta(TOPIC_COUNT)
    SEED: int = 0x0D15EA5E
    CHUNK_LEN: int = 0              # tokens per sampler chunk; 0 = auto from the global token count (32..128)
    EVAL_EVERY: int = 0             # log-likelihood every N sweeps (0 = only at the end)
    CKPT_EVERY: int = 0             # checkpoint every N sweeps (0 = never)
    # paths
    LPATH: str = "./oni_data"       # local results / feedback directory (per source subdirs)
    HPATH: str = ""                 # unused (no HDFS); kept for duxbay.conf compatibility
    DATA_ROOT: str = "./oni_store"  # columnar day store
    TOP_DOMAINS: str = ""           # top-1M list (Alexa-style CSV: rank,domain)
    PUBLIC_SUFFIX: str = ""         # public suffix list (Mozilla PSL format); "" = built-in oni355/data list
    # OA
    IPLOC: str = ""                 # geo ip-range CSV
    NETWORK_CONTEXT: str = ""       # network context CSV
    extra: dict = field(default_factory=dict)

    def alpha(self) -> float:
        return self.ALPHA if self.ALPHA > 0 else 50.0 / self.TOPIC_COUNT

    def replace(self, **kw) -> "OniConfig":
        return dataclasses.replace(self, **kw)


_FIELDS = {f.name: f for f in dataclasses.fields(OniConfig) if f.name != "extra"}


def _coerce(name: str, value: str):
    f = _FIELDS[name]
    t = f.type if isinstance(f.type, type) else {"int": int, "float": float, "str": str}.get(str(f.type), str)
    if t is int:
        return int(float(value)) if re.fullmatch(r"[-+]?\d+(\.0*)?([eE]\d+)?", value.strip()) else int(value, 0)
    if t is float:
        return float(value)
    return value


def parse_duxbay(text: str) -> dict:
    """Parse bash-style KEY=VALUE lines (quotes stripped, ${VAR} expanded from earlier keys)."""
    out: dict[str, str] = {}
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        if line.startswith("export "):
            line = line[7:].strip()
        m = re.match(r"([A-Za-z_][A-Za-z0-9_]*)=(.*)$", line)
        if not m:
            continue
        key, val = m.group(1), m.group(2).strip()
        try:
            parts = shlex.split(val, comments=True)
            val = parts[0] if parts else ""
        except ValueError:
            val = val.strip("'\"")
        val = re.sub(r"\$\{?([A-Za-z_][A-Za-z0-9_]*)\}?", lambda mm: out.get(mm.group(1), ""), val)
        out[key] = val
    return out


def load_config(path: str | None = None, env: dict | None = None, **overrides) -> OniConfig:
    cfg = OniConfig()
    vals: dict = {}
    if path:
        with open(path) as f:
            vals.update(parse_duxbay(f.read()))
    env = os.environ if env is None else env
    for k, v in env.items():
        if k.startswith("ONI_") and k[4:] in _FIELDS:
            vals[k[4:]] = v
    extra = {}
    for k, v in vals.items():
        if k in _FIELDS:
            setattr(cfg, k, _coerce(k, v))
        else:
            extra[k] = v
    for k, v in overrides.items():
        if v is None:
            continue
        if k not in _FIELDS:
            raise KeyError(f"unknown config key {k}")
        setattr(cfg, k, v)
    cfg.extra = extra
    return cfg


def parse_lda_settings(text: str) -> dict:
    """lda-c settings.txt: ``var max iter N`` / ``var convergence X`` / ``em max iter N`` /
    ``em convergence X`` / ``alpha fixed|estimate``; plus our Gibbs keys (``sweeps``, ``burnin``,
    ``beta``, ``seed``, ``eval every``)."""
    out: dict = {"var_max_iter": 20, "var_convergence": 1e-6, "em_max_iter": 100, "em_convergence": 1e-4,
                 "estimate_alpha": True}
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        toks = line.split()
        key, val = " ".join(toks[:-1]).lower(), toks[-1]
        if key == "var max iter":
            out["var_max_iter"] = int(val)
        elif key == "var convergence":
            out["var_convergence"] = float(val)
        elif key == "em max iter":
            out["em_max_iter"] = int(val)
        elif key == "em convergence":
            out["em_convergence"] = float(val)
        elif key == "alpha":
            out["estimate_alpha"] = val.lower() == "estimate"
        elif key in ("sweeps", "burnin", "seed", "eval every"):
            out[key.replace(" ", "_")] = int(val)
        elif key == "beta":
            out["beta"] = float(val)
    return out
