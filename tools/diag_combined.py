#!/usr/bin/env python3
"""Step-by-step replay of bench/combined.py's setup (flow K=100, then DNS K=100) with a sync and a
progress line after every stage, and periodic Python stack dumps: locates a setup stall."""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.dump_traceback_later(20, repeat=True)
import torch  # noqa: E402

from oni355.parallel import comm as pc  # noqa: E402
from oni355.pipeline import common, dns as src  # noqa: E402
from oni355.pipeline.synthetic import build_source  # noqa: E402
from oni355.synth.dns import generate_dns  # noqa: E402

K = int(os.environ.get("DIAG_K", "100"))
FLOWS = int(os.environ.get("DIAG_FLOWS", "12500000"))
NDNS = int(os.environ.get("DIAG_DNS", "6250000"))
t0 = time.perf_counter()


def p(msg):
    torch.cuda.synchronize()
    print(f"[diag {time.perf_counter() - t0:7.1f}s] {msg}", flush=True)


comm = pc.init_from_env("cuda")
if FLOWS:
    fsu = build_source("flow", FLOWS, K, comm, seed=7)
    p(f"flow built {fsu.run.corpus.stats()}")
    fsu.model.initialize()
    p("flow init")
    fsu.day = None
day = generate_dns(NDNS, seed=7, rank=0, n_clients=max(32, NDNS // 40))
p("dns generated")
d = src.to_device(day.cols, comm.device)
p("dns to_device")
ts = src.top_set(day.top_domains)
p("top set")
words, _, _ = src.featurize(d, comm, ts, "intel")
p("dns featurized")
sides = [(common.u32_to_i64(d["ip_dst"]), words.to(torch.int64))]
vocab = common.global_vocab(sides[0][1], comm)
p(f"vocab {vocab.numel()}")
run = common.build_and_train(sides[0][0], sides[0][1], None, vocab, K, None, 0.01, 0x0D15EA5E, 0, 0, comm,
                             train=False)
p(f"dns corpus {run.corpus.stats()} maxlen {run.corpus.max_doc_len()}")
run.model.initialize()
p("dns init")
run.model.sweep(4)
p("dns 4 sweeps")
if FLOWS:
    fsu.model.sweep(4)
    p("flow 4 sweeps")
faulthandler.cancel_dump_traceback_later()
