"""Public-suffix rules for registered-domain extraction (K04).

The reference's DomainProcessor split a DNS name into subdomain / registered domain / TLD with a
country-code-aware rule ([U-M]). Here the rule set is data: a file in the Mozilla Public Suffix
List format (``//`` comments, ``*.`` wildcards, ``!`` exceptions), by default the curated
``oni355/data/public_suffix_list.dat``; ``PUBLIC_SUFFIX`` / ``ONI_PUBLIC_SUFFIX`` names a full
list instead. Rules become two open-addressing sets of FNV-1a hashes (rules incl. wildcard rules
stored as ``*.rest``; exceptions without the ``!``) that the device kernel probes
(csrc/kernels/strings.hip) and the oracle below replays bit for bit.

Matching (PSL algorithm): for k = min(labels, MAX_LABELS) … 1, the k-label suffix S_k is
  * an exception      → the public suffix is S_{k-1};
  * a rule, or ``*.`` + S_{k-1} is a rule → the public suffix is S_k;
the first k that decides wins; no rule → the public suffix is the last label (the ``*`` rule).
The registered domain is the public suffix plus one more label (the whole name when the name is
itself a public suffix).
"""
from __future__ import annotations

import os

from . import strings_spec as ss

DEFAULT_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data",
                            "public_suffix_list.dat")
MAX_LABELS = 6  # the kernel looks at most this many labels deep (rules in the PSL have ≤ 5)


class SuffixRules:
    def __init__(self, rules: list[str], exceptions: list[str]):
        self.rules = [r.lower() for r in rules]
        self.exceptions = [e.lower() for e in exceptions]
        self.rule_set = ss.HashSet([ss.fnv1a(r.encode()) for r in self.rules] or [1])
        self.exc_set = ss.HashSet([ss.fnv1a(e.encode()) for e in self.exceptions] or [1])
        self.max_labels = min(MAX_LABELS, max([r.count(".") + 1 for r in self.rules + self.exceptions] + [1]) + 1)

    @staticmethod
    def parse(text: str) -> "SuffixRules":
        rules, exc = [], []
        for raw in text.splitlines():
            line = raw.strip().split()[0] if raw.strip() else ""
            if not line or line.startswith("//"):
                continue
            line = line.encode("idna").decode("ascii") if not line.isascii() else line
            if line.startswith("!"):
                exc.append(line[1:])
            else:
                rules.append(line)
        return SuffixRules(rules, exc)

    @staticmethod
    def load(path: str | None = None) -> "SuffixRules":
        path = path or os.environ.get("ONI_PUBLIC_SUFFIX") or DEFAULT_PATH
        with open(path, encoding="utf-8") as f:
            return SuffixRules.parse(f.read())


_DEFAULT: SuffixRules | None = None


def default_rules() -> SuffixRules:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = SuffixRules.load()
    return _DEFAULT


def registered_start(name: bytes, b: int, rules: SuffixRules | None = None) -> int:
    """Start offset of the registered domain of name[:b] (trailing dots already stripped)."""
    rules = rules or default_rules()
    dots = [j for j in range(b - 1, -1, -1) if name[j] == 46][: rules.max_labels]
    nlab = len(dots) + 1 if b > 0 else 0

    def start(k: int) -> int:  # first byte of the k-label suffix
        return dots[k - 1] + 1 if k <= len(dots) else 0

    ps = 1
    for k in range(min(nlab, rules.max_labels), 0, -1):
        sk = name[start(k):b]
        if ss.fnv1a(sk) in rules.exc_set:
            ps = k - 1
            break
        if ss.fnv1a(sk) in rules.rule_set or (k >= 2 and ss.fnv1a(b"*." + name[start(k - 1):b]) in rules.rule_set):
            ps = k
            break
    if nlab <= ps:
        return 0
    return start(ps + 1)
