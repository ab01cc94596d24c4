"""Bench-scale checks on the MI355X (kernel tests alone use small inputs): the 12.5M-flow
day of the headline benchmark, sampled with ONI_CHECK_INVARIANTS=1 so every count invariant
(Σn_wk = Σn_k = tokens, n_k = column sums, Σn_dk = local tokens, no negative or padding counts)
is verified after every sweep() call, across the recount → delta switch, plus the numerical
health check and the planted anomalies' recall."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_bench_day_invariants_and_recall(gpu, monkeypatch):
    monkeypatch.setenv("ONI_CHECK_INVARIANTS", "1")
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    n = 12_500_000
    day = generate_flows(n, seed=7, n_hosts=n // 25)
    res = run_flow(day.cols, K=20, sweeps=40, maxresults=3000, device="cuda:0", eval_every=4)
    m = res.lda.model
    assert m.cfg.check_invariants and m.sweeps_done == 40
    assert m._delta_on, "the sampler never switched to the delta count mode at bench scale"
    ll = [v for _, v in m.likelihoods]
    assert len(ll) == 10 and all(np.isfinite(ll)) and ll[-1] > ll[0]
    hits = np.isin(day.anomaly_rows, res.rows)
    assert hits.mean() >= 0.9, hits.mean()
