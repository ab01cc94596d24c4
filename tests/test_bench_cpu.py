"""bench.py contract on CPU (gloo): one JSON line from rank 0 with the BASELINE metric/config keys,
for world size 1 and for a 2-rank torch.distributed.run launch (the driver's N>1 command shape)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "2", "--warmup", "1", "--flows-per-gpu", "3000", "--sweeps", "6", "--device", "cpu"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # stdout is exactly the JSON line
    return json.loads(lines[0])


def _check(out, n):
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert out["metric"] == base["metric"]
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["higher_is_better"] is True
    assert out["scaling"] == "weak" and out["config"]["parallelism"] == f"dp{n}"
    assert out["config"]["global_batch"] == 3000 * n
    # a step is a full day run: every stage is timed and the in-step training reports its sweep rate
    for stage in ("h2d_s", "featurize_s", "vocab_s", "corpus_s", "init_s", "train_s", "score_prep_s", "score_s",
                  "results_s", "step_s"):
        assert stage in out["stage_median_s"], stage
    assert out["gibbs_iters_per_sec"] > 0 and out["config"]["sweeps_per_step"] == 6
    assert out["vs_baseline"] is None
    # the realistic-vocabulary day of the same shape is reported next to the headline
    rv = out["realistic_vocab"]
    assert rv["value"] > 0 and rv["steps"] == 3 and rv["vocab"] > 0 and 0.0 <= rv["planted_anomaly_recall_topN"] <= 1.0


def test_bench_single_process():
    _check(_run([sys.executable, "bench.py", *ARGS]), 1)


def test_bench_self_launches_ranks():
    """``bench.py --gpus 2`` outside torchrun starts its own 2-rank torch.distributed.run child."""
    _check(_run([sys.executable, "bench.py", "--gpus", "2", *ARGS]), 2)


@pytest.mark.slow
def test_bench_two_ranks_torchrun():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "bench.py", "--gpus", "2", *ARGS]
    _check(_run(cmd), 2)


def test_allreduce_bench_gloo_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "bench/allreduce.py", "--device", "cpu",
           "--min-kb", "64", "--max-mb", "1", "--iters", "2", "--warmup", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert [x["bytes"] for x in rows] == [65536, 262144, 1048576]
    assert all(x["ok"] and x["ranks"] == 2 and x["busbw_GBps"] > 0 for x in rows)


def test_combined_bench_cpu_and_sizing():
    from oni355.utils import sizing
    small = ["--device", "cpu", "--flows-per-gpu", "2000", "--dns-per-gpu", "1000", "--proxy-per-gpu", "1000",
             "--steps", "1", "--warmup", "1", "--topics", "50"]
    out = _run([sys.executable, "bench/combined.py", *small, "--mode", "sweep"])
    assert out["value"] > 0 and set(out["ms_per_sweep_by_model"]) == {"flow", "dns", "proxy"}
    assert out["tokens"] == {"flow": 4000, "dns": 1000, "proxy": 1000}
    assert out["projection_1B_events_8gpu"]["fits_288GB"] is True
    # day mode (the default): every source's whole day per step, result rows written
    day = _run([sys.executable, "bench/combined.py", *small, "--sweeps", "4", "--maxresults", "50"])
    assert day["value"] > 0 and set(day["day_s_by_model"]) == {"flow", "dns", "proxy"}
    assert {k: v["tokens"] for k, v in day["model_stats"].items()} == {"flow": 4000, "dns": 1000, "proxy": 1000}
    assert all(v["rows"] == 50 for v in day["model_stats"].values())
    # the planner grows with every input and flags what cannot fit
    a = sizing.plan("flow", 10**6, 20, 10**4, 10**4)
    b = sizing.plan("flow", 2 * 10**6, 20, 10**4, 10**4)
    assert b.steady_bytes > a.steady_bytes and b.peak_bytes > b.steady_bytes
    assert not sizing.plan("flow", 20 * 10**9, 100, 10**6, 10**6).fits()


def test_bench_forced_one_rank_process_group_matches_plain():
    """ONI_FORCE_DIST=1 drives every collective through a real 1-rank process group (the RCCL code
    path on a single GPU box; gloo here): same model and results as the collective-free run."""
    plain = _run([sys.executable, "bench.py", *ARGS])
    env_cmd = [sys.executable, "bench.py", *ARGS]
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1", ONI_FORCE_DIST="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    r = subprocess.run(env_cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    forced = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    _check(forced, 1)
    for k in ("loglik", "tokens", "vocab", "docs_local", "planted_anomaly_recall_topN"):
        assert forced[k] == plain[k], k
    assert forced["allreduce_bytes_per_sweep"] > 0 and plain["allreduce_bytes_per_sweep"] == 0


def test_sizing_counts_mh_burn_in_and_posterior_sums():
    """The K = 100 projection includes the MH word tables, the dense burn-in's second corpus and
    model, the posterior sums and θ / φ: the 1B-token flow model on one MI355X measured 154 GB
    (profiles/r5/combined_flow_1B_tokens_k100_1gpu.json); the round-4 formula said 68 GB."""
    from oni355.utils import sizing
    p = sizing.plan("flow", 500_000_000, 100, 20_000_000, 7008)
    assert 0.75 * 154e9 < p.peak_bytes < 1.25 * 154e9, p.as_dict()
    nb = sizing.plan("flow", 500_000_000, 100, 20_000_000, 7008, mh_burn=0)
    assert nb.peak_bytes < p.peak_bytes


def test_day_ab_alternates_variants_on_one_day(tmp_path):
    """bench/day_ab.py (the in-process whole-day A/B): every variant runs every round on the same
    generated day; an env-only variant draws the same chain as the base (same log-likelihood)."""
    out = tmp_path / "ab.json"
    cmd = [sys.executable, "bench/day_ab.py", "--device", "cpu", "--flows", "3000", "--topics", "20",
           "--sweeps", "6", "--rounds", "2", "--variant", "base:", "--variant", "ab:ONI_SAMPLER_AB=32",
           "--variant", "L64:chunk=64", "--out", str(out)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(out.read_text())
    assert set(d["summary"]) == {"base", "ab", "L64"} and all(len(v) == 2 for v in d["days"].values())
    assert d["variants"]["L64"]["chunk"] == 64 and d["variants"]["ab"]["env"] == {"ONI_SAMPLER_AB": "32"}
    ll = {n: {x["loglik"] for x in v} for n, v in d["days"].items()}
    assert ll["base"] == ll["ab"] and len(ll["base"]) == 1  # CPU oracle: the A/B bits change no draw
