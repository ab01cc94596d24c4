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
