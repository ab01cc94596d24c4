"""Long-tail synthetic vocabularies (bench --realistic-vocab)."""
import torch

from oni355.pipeline import dns as D
from oni355.pipeline import proxy as P
from oni355.synth.dns import generate_dns
from oni355.synth.proxy import generate_proxy


def _words_dns(wide, n=100_000):
    d = generate_dns(n, seed=3, wide_vocab=wide)
    return D.featurize(D.to_device(d.cols, "cpu"), None, D.top_set(d.top_domains), "intel")[0]


def _words_proxy(wide, n=100_000):
    p = generate_proxy(n, seed=3, wide_vocab=wide)
    return P.featurize(p.cols, "cpu", None, P.top_set(None))[0]


def test_wide_vocab_grows_dns_and_proxy_vocabularies():
    """The long tail is a codebook of recurring, client-owned behaviours: the vocabulary grows
    while day-unique words stay a tiny share of the rows (the planted rows stay findable). DNS and
    proxy words are quantised features (quintiles, deciles, codes), so their vocabularies grow
    less than the flow day's port-keyed one (100k rows: DNS 2.2k -> 2.5k, proxy 1.5k -> 2.3k)."""
    for fn, grow in ((_words_dns, 1.1), (_words_proxy, 1.3)):
        base, wide = fn(0.0), fn(0.5)
        assert torch.unique(wide).numel() > grow * torch.unique(base).numel()
        _, cnt = torch.unique(wide, return_counts=True)
        assert int((cnt == 1).sum()) < 0.005 * wide.numel()


def test_wide_vocab_keeps_anomalies_and_shapes():
    d = generate_dns(5_000, seed=4, wide_vocab=0.5)
    assert len(d.cols["dns_qry_name"]) == 5_000 and d.anomaly_rows.size
    names = d.cols["dns_qry_name"]
    assert all(names[int(i)].endswith("tunnel.biz") for i in d.anomaly_rows)
    p = generate_proxy(5_000, seed=4, wide_vocab=0.5)
    assert all(p.cols["host"][int(i)].endswith("badcdn-sync.biz") for i in p.anomaly_rows)
