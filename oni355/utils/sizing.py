"""HBM sizing for one GPU's share of a day (288 GB HBM3E per MI355X).

Byte counts follow the device layout of this engine:

* tokens (per token): SELL word id 4 B + topic 1 B + word-sorted position 4 B + word-sorted word
  id 4 B + word-sorted slot 4 B + (old|new) topic pair 2 B + change bit 1/8 B  ≈ 19.1 B;
* documents (per doc): two n_dk rows (ping-pong) of KS int32 + CSR/chunk tables ≈ 8·KS + 40 B;
* vocabulary (per word): n_wk + q + two Δ buffers, KS × 4 B each  = 16·KS B;
* raw columns on device while featurizing (per event): flow 9 columns ≈ 44 B, DNS/proxy ≈ 40 B plus
  string bytes;
* corpus build transient: the (doc, word) pair sort holds ≈ 24 B per token at its peak;
* posterior-average sums (the last quarter of the chain): n_dk / n_wk sums of KS entries per doc /
  word, int64 when S times the largest count can pass 2^31 (config-4/5 magnitudes), int32 below;
* scoring: θ (docs × KS f32) and φ (vocab × KS f32);
* MH models (K ≥ 100): the word proposal tables (alias records V·K·16 B + sums, or 64-B CDF rows
  when 3·V·K > 2·T) and, during the dense burn-in, a second corpus of the dense tiling with its own
  document and word tables (the round-4 estimate left these out and projected 68 GB for
  the 1B-token flow model that measured 154 GB, profiles/r5/combined_flow_1B_tokens_k100_1gpu.json).

``plan()`` returns the estimate; ``bench/combined.py`` prints it next to torch's measured peak.
"""
from __future__ import annotations

from dataclasses import dataclass

HBM_BYTES = 288 * 10**9

TOKEN_BYTES = 4 + 1 + 4 + 4 + 4 + 2 + 1 / 8
BUILD_BYTES_PER_TOKEN = 24
RAW_BYTES = {"flow": 44, "dns": 40, "proxy": 40}
TOKENS_PER_EVENT = {"flow": 2, "dns": 1, "proxy": 1}


def ks_of(K: int) -> int:
    from ..models.gibbs import tiling_for
    G, KP = tiling_for(K)
    return G * KP


@dataclass
class Plan:
    source: str
    events: int
    tokens: int
    docs: int
    vocab: int
    K: int
    steady_bytes: int
    peak_bytes: int

    def fits(self, hbm: int = HBM_BYTES, headroom: float = 0.9) -> bool:
        return self.peak_bytes <= hbm * headroom

    def as_dict(self) -> dict:
        return {"source": self.source, "events": self.events, "tokens": self.tokens, "docs": self.docs,
                "vocab": self.vocab, "K": self.K, "steady_GB": round(self.steady_bytes / 1e9, 3),
                "peak_GB": round(self.peak_bytes / 1e9, 3)}


def plan(source: str, events: int, K: int, docs: int, vocab: int, string_bytes_per_event: int = 0,
         samples: int = 50, mh_burn: int | None = None, tokens_global: int | None = None) -> Plan:
    """Estimate one GPU's HBM use for ``events`` local events of ``source`` (``samples`` posterior
    samples; ``mh_burn``: dense burn-in sweeps of an MH model, default ONI_MH_BURN's 20;
    ``tokens_global``: the model's token count over all GPUs, default the local one)."""
    from ..models.gibbs import sampler_for, tiling_for
    KS = ks_of(K)
    tokens = events * TOKENS_PER_EVENT[source]
    T = tokens_global or tokens
    steady = int(tokens * TOKEN_BYTES + docs * (8 * KS + 40) + vocab * 16 * KS)
    # posterior sums: a doc row / word row / topic total of S samples, int64 past 2^31
    wide = lambda bound: 8 if bound * samples > 2**31 - 1 else 4  # noqa: E731
    sums = docs * KS * wide(tokens // max(docs, 1) * 64) + vocab * KS * wide(T // max(vocab, 1) * 64)
    scoring = (docs + vocab) * KS * 4
    extra = 0
    if sampler_for(K) == "mh":
        cdf = 3 * vocab * K > 2 * T or 16 * vocab * K > 128e6  # models/gibbs.py _setup_mh
        extra += vocab * 64 if cdf else vocab * (K * 16 + 4)
        burn = 20 if mh_burn is None else mh_burn
        if burn > 0:
            Gd, KPd = tiling_for(K, "dense")
            KSd = Gd * KPd
            extra += int(tokens * TOKEN_BYTES + docs * (8 * KSd + 40) + vocab * 16 * KSd)
    raw = events * (RAW_BYTES[source] + string_bytes_per_event)
    peak = steady + sums + scoring + extra + raw + tokens * BUILD_BYTES_PER_TOKEN
    return Plan(source, events, tokens, docs, vocab, K, steady, int(peak))


def plan_combined(events_total: int, gpus: int, K: int = 100, mix=(0.5, 0.25, 0.25),
                  vocab=(1_000_000, 1_000_000, 1_000_000)) -> list[Plan]:
    """Config 5 (flow + DNS + proxy, ``events_total`` events, ``gpus`` GPUs, one model per source):
    per-GPU plans, docs ≈ events/25 (flow) or /40 (DNS, proxy) as in the synthetic generators."""
    out = []
    for src, frac, V, per_doc in zip(("flow", "dns", "proxy"), mix, vocab, (25, 40, 40)):
        ev = int(events_total * frac) // gpus
        out.append(plan(src, ev, K, docs=max(1, ev // per_doc), vocab=V,
                        string_bytes_per_event=0 if src == "flow" else 48))
    return out
