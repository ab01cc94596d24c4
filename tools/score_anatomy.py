#!/usr/bin/env python3
"""Why does a flow rank where it ranks? For the top rows of a (realistic-vocabulary) flow day and
for its planted anomalies, print both endpoint scores with their decomposition: the word, its day
count, the document's size, θ's largest entry and θ on the word's main topic (diagnostics for the
recall work in docs/performance.md).

  python tools/score_anatomy.py 12500000 cuda [--narrow]
"""
import sys, os, numpy as np, collections, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oni355.synth.flow import generate_flows
from oni355.pipeline import flow as fp
from oni355.ref import spec
n = int(sys.argv[1]); dev = sys.argv[2] if len(sys.argv) > 2 else "cpu"
wide = "--narrow" not in sys.argv
day = generate_flows(n, seed=7, n_hosts=max(64, n // 25), wide_vocab=wide)
res = fp.run_flow(day.cols, K=20, sweeps=200 if dev != "cpu" else 60, maxresults=n, device=dev)
run = res.lda; m = run.model
nwk = m.nwk[:, :20].cpu().numpy(); ndk = m.ndk_cur[:, :20].cpu().numpy()
vocab = run.vocab.cpu().numpy(); dkeys = run.doc_keys64.cpu().numpy()
theta = m.theta()[:, :20].cpu().numpy(); phi = m.q[:, :20].cpu().numpy()
nk = nwk.sum(0)
order = np.asarray(res.rows)
rank = np.empty(n, np.int64); rank[order] = np.arange(order.size)
print("nk mean", nk.mean(), "V", vocab.size)
def info(i):
    r = order[i]
    out = []
    for side, doc, w, s in (("src", day.cols["sip"][r], res.src_words[i], res.src_scores[i]), ("dst", day.cols["dip"][r], res.dst_words[i], res.dst_scores[i])):
        di = np.searchsorted(dkeys, int(doc)); wi = np.searchsorted(vocab, int(w))
        kk = np.argmax(nwk[wi])
        out.append(f"{side}: {spec.flow_word_str(int(w))} wc={nwk[wi].sum()} wtop={nwk[wi].max()} nd={ndk[di].sum()} thmax={theta[di].max():.3f} th[wk]={theta[di,kk]:.4f} s*nk={s*nk.mean():.4f}")
    return " | ".join(out)
for i in range(40):
    print(i, "planted" if order[i] in set(day.anomaly_rows.tolist()) else "", info(i))
for r in sorted(day.anomaly_rows.tolist(), key=lambda r: -rank[r])[:30]:
    print("A", rank[r], info(rank[r]))
