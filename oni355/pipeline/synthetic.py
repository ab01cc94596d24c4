"""Synthetic-day setup shared by the benchmarks: generate one rank's shard of a day of one source,
featurize it on the device, and build (but do not train) its LDA run.

Weak scaling: every rank generates ``per_rank`` events with its own RNG stream
(``rank`` offsets the generator seed), and the population (hosts / clients) scales with the
node-wide day, so N ranks together form one N×-sized day.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from ..parallel.comm import Comm
from . import common


@dataclass
class SourceSetup:
    source: str
    K: int
    per_rank: int
    n_total: int
    day: object            # generator output (cols, anomaly_rows, ...)
    sides: list            # [(doc_keys64, word_keys64)] per event endpoint
    vocab: torch.Tensor
    run: common.LdaRun

    @property
    def model(self):
        return self.run.model


def build_source(source: str, per_rank: int, K: int, comm: Comm, seed: int = 7, chunk_len: int = 0,
                 lda_seed: int = 0x0D15EA5E) -> SourceSetup:
    dev, rank, world = comm.device, comm.rank, comm.world
    n_total = per_rank * world
    if source == "flow":
        from . import flow
        from ..synth.flow import generate_flows
        day = generate_flows(per_rank, seed=seed, rank=rank, n_hosts=max(64, n_total // 25))
        d = flow.to_device(day.cols, dev)
        cuts = flow.compute_cuts(d, comm)
        sw, dw = flow.wordify(d, cuts)
        sides = [(common.u32_to_i64(d["sip"]), common.u32_to_i64(sw)), (common.u32_to_i64(d["dip"]), common.u32_to_i64(dw))]
    elif source == "dns":
        from . import dns as src
        from ..synth.dns import generate_dns
        day = generate_dns(per_rank, seed=seed, rank=rank, n_clients=max(32, n_total // 40))
        d = src.to_device(day.cols, dev)
        words, _, _ = src.featurize(d, comm, src.top_set(day.top_domains), "intel")
        sides = [(common.u32_to_i64(d["ip_dst"]), words.to(torch.int64))]
    elif source == "proxy":
        from . import proxy as src
        from .dns import top_set
        from ..synth.dns import top_domain_list
        from ..synth.proxy import generate_proxy
        day = generate_proxy(per_rank, seed=seed, rank=rank, n_clients=max(32, n_total // 40))
        words, _, _ = src.featurize(day.cols, dev, comm, top_set(top_domain_list()))
        from ..io import staging
        doc = staging.upload(np.asarray(day.cols["clientip"], np.uint32).astype(np.int64), dev)
        sides = [(doc, words.to(torch.int64))]
    else:
        raise ValueError(f"unknown source {source}")
    doc_keys = torch.cat([s[0] for s in sides])
    word_keys = torch.cat([s[1] for s in sides])
    vocab = common.global_vocab(word_keys, comm)
    run = common.build_and_train(doc_keys, word_keys, None, vocab, K, None, 0.01, lda_seed, 0, chunk_len, comm,
                                 train=False)
    return SourceSetup(source, K, per_rank, n_total, day, sides, vocab, run)
