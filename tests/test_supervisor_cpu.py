"""``oni-ml --max-restarts``: a supervised run survives a crashed / numerically corrupted child by
starting a fresh child that resumes from the last checkpoint, and its results are bitwise equal
to an uninterrupted run (SURVEY.md §5.3 failure detection + §5.4 checkpoint/resume)."""
import os
import subprocess
import sys

import pytest

from oni355.cli import ml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _args(lp, conf):
    return ["20160708", "flow", "1.0", "60", "--synthetic", "5000", "--device", "cpu", "--sweeps", "12",
            "--lpath", lp, "--quiet", "--config", conf]


def _read(lp):
    with open(os.path.join(lp, "flow", "20160708", "flow_results.csv"), "rb") as f:
        return f.read()


@pytest.mark.parametrize("kind", ["exit", "nan"])
def test_supervised_run_recovers_bitwise(tmp_path, kind):
    conf = str(tmp_path / "none.conf")
    plain = str(tmp_path / "plain")
    assert ml.main(_args(plain, conf)) == 0
    sup = str(tmp_path / "sup")
    env = dict(os.environ, ONI_FAULT=f"rank:0,sweep:6,kind:{kind},attempt:0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "oni355.cli.ml", *_args(sup, conf), "--max-restarts", "2",
                        "--ckpt-every", "4"], env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "attempt 0 failed" in r.stderr and "restarting from the last checkpoint" in r.stderr
    assert _read(plain) == _read(sup)
    # the supervisor's own checkpoint directory is removed after success
    assert not os.path.exists(os.path.join(sup, "flow", "20160708", ".ckpt"))


def test_supervisor_gives_up_after_max_restarts(tmp_path):
    conf = str(tmp_path / "none.conf")
    env = dict(os.environ, ONI_FAULT="rank:0,sweep:2,kind:exit", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "oni355.cli.ml", *_args(str(tmp_path / "x"), conf),
                        "--max-restarts", "1", "--ckpt-every", "4"], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 17
    assert "attempt 1 failed (exit 17); giving up" in r.stderr


def test_burnin_gates_likelihood_trace(tmp_path):
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    day = generate_flows(3000, seed=5)
    a = run_flow(day.cols, K=20, sweeps=12, maxresults=20, device="cpu", eval_every=2)
    b = run_flow(day.cols, K=20, sweeps=12, maxresults=20, device="cpu", eval_every=2, burnin=6)
    assert [s for s, _ in a.lda.model.likelihoods] == [2, 4, 6, 8, 10, 12]
    assert [s for s, _ in b.lda.model.likelihoods] == [8, 10, 12]
    assert a.lda.model.likelihoods[-1] == b.lda.model.likelihoods[-1]
