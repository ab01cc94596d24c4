"""ONI_CHAINS: several independent Gibbs chains over one corpus, scored by the average of their
pair scores (pipeline.common.LdaRun.pair_scores) -- deterministic, the same total sweep count, and
different from the single-chain ranking."""
import numpy as np
import pytest

from oni355.pipeline.flow import run_flow
from oni355.synth.flow import generate_flows


def _run(monkeypatch, chains):
    monkeypatch.setenv("ONI_CHAINS", str(chains))
    day = generate_flows(6000, seed=5)
    return run_flow(day.cols, K=20, sweeps=16, maxresults=200, device="cpu"), day


def test_two_chains_average_scores(monkeypatch):
    one, day = _run(monkeypatch, 1)
    two, _ = _run(monkeypatch, 2)
    again, _ = _run(monkeypatch, 2)
    assert len(two.lda.extra_models) == 1 and two.timings["chains"] == 2
    assert two.lda.model.sweeps_done == 8 and two.lda.extra_models[0].sweeps_done == 8
    assert np.array_equal(two.rows, again.rows) and np.array_equal(two.scores, again.scores)
    assert not np.array_equal(one.scores, two.scores)
    assert np.all(np.diff(two.scores) >= 0)
    assert np.isin(day.anomaly_rows, two.rows).mean() >= np.isin(day.anomaly_rows, one.rows).mean() - 0.2


def test_branching_chains_share_the_burn_in(monkeypatch):
    """ONI_CHAIN_BRANCH = B: both chains run the first B sweeps once (chain 1), the second starts
    from chain 1's state at sweep B with its own seed; the total sweep count stays the budget."""
    import torch
    monkeypatch.setenv("ONI_CHAIN_BRANCH", "6")
    two, day = _run(monkeypatch, 2)
    again, _ = _run(monkeypatch, 2)
    m1, m2 = two.lda.model, two.lda.extra_models[0]
    assert m1.sweeps_done == m2.sweeps_done == 6 + (16 - 6) // 2
    assert two.timings["chain_branch"] == 6 and two.timings["sweeps"] == 16
    assert np.array_equal(two.rows, again.rows) and np.array_equal(two.scores, again.scores)
    assert not torch.equal(m1.canonical_z(), m2.canonical_z())  # the branches diverged
    m2.check_invariants()
