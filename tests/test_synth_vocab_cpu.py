"""Long-tail synthetic vocabularies (bench --realistic-vocab)."""
import torch

from oni355.pipeline import dns as D
from oni355.pipeline import proxy as P
from oni355.synth.dns import generate_dns
from oni355.synth.proxy import generate_proxy


def _v_dns(wide):
    d = generate_dns(20_000, seed=3, wide_vocab=wide)
    return torch.unique(D.featurize(D.to_device(d.cols, "cpu"), None, D.top_set(d.top_domains), "intel")[0]).numel()


def _v_proxy(wide):
    p = generate_proxy(20_000, seed=3, wide_vocab=wide)
    return torch.unique(P.featurize(p.cols, "cpu", None, P.top_set(None))[0]).numel()


def test_wide_vocab_grows_dns_and_proxy_vocabularies():
    assert _v_dns(0.5) > 3 * _v_dns(0.0)
    assert _v_proxy(0.5) > 2 * _v_proxy(0.0)


def test_wide_vocab_keeps_anomalies_and_shapes():
    d = generate_dns(5_000, seed=4, wide_vocab=0.5)
    assert len(d.cols["dns_qry_name"]) == 5_000 and d.anomaly_rows.size
    names = d.cols["dns_qry_name"]
    assert all(names[int(i)].endswith("tunnel.biz") for i in d.anomaly_rows)
    p = generate_proxy(5_000, seed=4, wide_vocab=0.5)
    assert all(p.cols["host"][int(i)].endswith("badcdn-sync.biz") for i in p.anomaly_rows)
