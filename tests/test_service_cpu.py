"""oni-mld (oni355/cli/service.py): a forwarded oni-ml day runs in the resident service, the client
never imports torch, and the results equal a local run's; with no service answering the client runs
the day itself."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CLIENT = ("import sys; from oni355.cli import ml; rc = ml.main(sys.argv[1:]); "
           "assert 'torch' not in sys.modules, 'client imported torch'; sys.exit(rc)")


def _args(lp):
    return ["20160708", "flow", "1.0", "40", "--synthetic", "4000", "--device", "cpu", "--sweeps", "4",
            "--lpath", lp, "--quiet"]


def _read(p):
    with open(p) as f:
        return f.read()


def test_forwarded_day_matches_local_run(tmp_path):
    sock = str(tmp_path / "mld.sock")
    env = dict(os.environ, PYTHONPATH=ROOT)
    srv = subprocess.Popen([sys.executable, "-m", "oni355.cli.service", "--socket", sock, "--max-requests", "2",
                            "--no-warm"], cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True)
    try:
        t0 = time.time()
        while not os.path.exists(sock):
            assert srv.poll() is None, srv.stderr.read()
            assert time.time() - t0 < 120
            time.sleep(0.05)
        remote = str(tmp_path / "remote")
        r = subprocess.run([sys.executable, "-c", _CLIENT, *_args(remote), "--service", sock], cwd=str(tmp_path),
                           env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        # a failing day reports its exit code and stderr through the socket, the service survives
        r2 = subprocess.run([sys.executable, "-c", _CLIENT, "20160708", "nosuchsource", "--service", sock],
                            cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
        assert r2.returncode == 2 and "nosuchsource" in r2.stderr
        srv.wait(timeout=60)
        assert srv.returncode == 0
    finally:
        if srv.poll() is None:
            srv.kill()
            srv.wait()
    local = str(tmp_path / "local")
    from oni355.cli import ml
    assert ml.main(_args(local)) == 0
    res = os.path.join("flow", "20160708", "flow_results.csv")
    assert _read(os.path.join(remote, res)) == _read(os.path.join(local, res))


def test_no_service_runs_locally(tmp_path):
    lp = str(tmp_path / "lp")
    env = dict(os.environ, PYTHONPATH=ROOT, ONI_MLD_SOCKET=str(tmp_path / "absent.sock"))
    r = subprocess.run([sys.executable, "-m", "oni355.cli.ml", *_args(lp)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert os.path.exists(os.path.join(lp, "flow", "20160708", "flow_results.csv"))


def test_service_declines_what_it_cannot_run(tmp_path, monkeypatch):
    """Import-time knobs set differently from the service's, supervised runs and multi-GPU runs come
    back as "run locally" (the client then runs the day in its own process)."""
    from oni355.cli import service
    monkeypatch.delenv("ONI_SPLIT_DEN", raising=False)
    rep = service._run_one({"argv": _args(str(tmp_path / "a")), "env": {"ONI_SPLIT_DEN": "4"}})
    assert rep["local"] and "ONI_SPLIT_DEN" in rep["stderr"]
    rep = service._run_one({"argv": _args(str(tmp_path / "b")) + ["--max-restarts", "1"], "env": {}})
    assert rep["local"] and "--max-restarts" in rep["stderr"]
    rep = service._run_one({"argv": _args(str(tmp_path / "c")) + ["--gpus", "2"], "env": {}})
    assert rep["local"] and "2 GPUs" in rep["stderr"]
    assert "ONI_MLD_INSIDE" not in os.environ  # the service's environment is restored
