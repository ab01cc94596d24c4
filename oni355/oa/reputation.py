"""Reputation services (oni-oa components/reputation: McAfee GTI, Facebook ThreatExchange;
SURVEY.md §2.2 C30, [U-M]) behind one plugin interface.

The target environment has no network, so the shipped implementation is an offline CSV-backed
service (``indicator,verdict`` rows: IPs, domains or URL prefixes); the networked services are
registered as plugins that raise a clear error when instantiated without connectivity/config.
"""
from __future__ import annotations

import csv
import json
import os


class ReputationService:
    name = "base"

    def check(self, keys: list[str]) -> dict[str, str]:  # pragma: no cover - interface
        raise NotImplementedError


class CsvReputation(ReputationService):
    """Offline indicator list: exact IP/domain match, or URL/domain suffix match."""

    name = "csv"

    def __init__(self, path: str):
        self.exact: dict[str, str] = {}
        with open(path, newline="") as f:
            for row in csv.reader(f):
                if row and not row[0].startswith("#"):
                    self.exact[row[0].strip().lower()] = row[1].strip() if len(row) > 1 else "listed"

    def check(self, keys: list[str]) -> dict[str, str]:
        out = {}
        for k in keys:
            kl = k.strip().lower()
            v = self.exact.get(kl)
            if v is None:
                host = kl.split("://", 1)[-1].split("/", 1)[0].split(":", 1)[0]
                parts = host.split(".")
                for i in range(len(parts) - 1):
                    v = self.exact.get(".".join(parts[i:]))
                    if v:
                        break
            out[k] = v or ""
        return out


class _NetworkService(ReputationService):
    config_key = ""

    def __init__(self, config_path: str):
        if not os.path.exists(config_path):
            raise FileNotFoundError(f"{self.name}: config {config_path} missing")
        with open(config_path) as f:
            self.config = json.load(f)
        raise RuntimeError(f"{self.name}: network reputation lookups are unavailable in this deployment "
                           "(no egress); use CsvReputation with an exported indicator list")


class GtiReputation(_NetworkService):
    name = "gti"


class FbThreatExchange(_NetworkService):
    name = "fb"


REGISTRY = {"csv": CsvReputation, "gti": GtiReputation, "fb": FbThreatExchange}


def load_services(spec: str | None) -> list[ReputationService]:
    """``"csv:/path/list.csv,gti:/path/gti.json"`` → instantiated services."""
    out: list[ReputationService] = []
    for part in (spec or "").split(","):
        if not part.strip():
            continue
        kind, _, arg = part.partition(":")
        out.append(REGISTRY[kind.strip()](arg.strip()))
    return out
