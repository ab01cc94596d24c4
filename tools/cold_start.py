#!/usr/bin/env python3
"""Cold single-day latency breakdown (verdict r3 item 8): wall time of fresh processes doing
progressively more of what a cold ``oni-ml YYYYMMDD flow`` config-2 day does, so the differences
name the cost of each layer (interpreter + torch import, HIP runtime init, our imports, kernel
library load, the day itself). Also runs the real CLI on a stored 1M-flow day, cold and forwarded to
a warm ``oni-mld`` service (oni355/cli/service.py).

  python tools/cold_start.py --flows 1000000
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = {
    "python": "pass",
    "import_torch": "import torch",
    "hip_init": "import torch; torch.zeros(1, device='cuda'); torch.cuda.synchronize()",
    "import_oni": "import torch; torch.zeros(1, device='cuda'); import oni355.pipeline.flow, oni355.pipeline.daily",
    "lib_load": ("import torch; torch.zeros(1, device='cuda'); import oni355.pipeline.flow; "
                 "from oni355.ops import _lib, native; _lib.lib(); native.lib()"),
    "first_kernels": ("import torch; torch.zeros(1, device='cuda'); import oni355.pipeline.flow as f; "
                      "from oni355.synth.flow import generate_flows; "
                      "f.run_flow(generate_flows(2000, seed=1).cols, K=20, sweeps=4, maxresults=10, device='cuda:0'); "
                      "torch.cuda.synchronize()"),
}


def wall(code: str, env) -> float:
    t = time.perf_counter()
    subprocess.run([sys.executable, "-c", code], check=True, env=env, cwd=ROOT, capture_output=True)
    return time.perf_counter() - t


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)
    out = {"steps_s": {}}
    for name, code in STEPS.items():
        out["steps_s"][name] = round(min(wall(code, env) for _ in range(a.reps)), 3)
    sys.path.insert(0, ROOT)
    from oni355.store import columnar
    from oni355.synth.flow import generate_flows
    tmp = tempfile.mkdtemp(prefix="oni_cold_")
    root, lp = os.path.join(tmp, "store"), os.path.join(tmp, "lp")
    columnar.write_day(root, "flow", "20160801", generate_flows(a.flows, seed=99, n_hosts=max(64, a.flows // 25)).cols)
    conf = os.path.join(tmp, "none.conf")
    cmd = [sys.executable, "-m", "oni355.cli.ml", "20160801", "flow", "1.0", "3000", "--data-root", root, "--lpath",
           lp, "--config", conf, "--device", "cuda", "--quiet"]
    walls = []
    for _ in range(a.reps):
        t = time.perf_counter()
        r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True)
        walls.append(time.perf_counter() - t)
        if r.returncode != 0:
            print(r.stderr[-3000:], file=sys.stderr)
            return 1
    rec = [json.loads(x) for x in open(os.path.join(lp, "flow", "20160801", "metrics.jsonl"))][-1]
    out["cli_config2_wall_s"] = round(min(walls), 3)
    out["cli_config2_walls"] = [round(w, 3) for w in walls]
    out["in_process"] = {k: rec.get(k) for k in ("load_s", "day_s", "featurize_s", "vocab_s", "corpus_s", "init_s",
                                                  "train_s", "score_s", "train_dev_s")}
    # the same command line forwarded to a resident service (started and warmed outside the clock)
    sock = os.path.join(tmp, "mld.sock")
    srv = subprocess.Popen([sys.executable, "-m", "oni355.cli.service", "--socket", sock, "--max-requests",
                            str(a.reps)], env=env, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    t0 = time.perf_counter()
    while not os.path.exists(sock):
        if srv.poll() is not None or time.perf_counter() - t0 > 300:
            print(srv.stderr.read().decode()[-3000:], file=sys.stderr)
            return 1
        time.sleep(0.02)
    out["service_warmup_s"] = round(time.perf_counter() - t0, 3)
    walls = []
    for _ in range(a.reps):
        t = time.perf_counter()
        r = subprocess.run(cmd + ["--service", sock], env=env, cwd=ROOT, capture_output=True, text=True)
        walls.append(time.perf_counter() - t)
        if r.returncode != 0:
            print(r.stderr[-3000:], file=sys.stderr)
            return 1
    srv.wait(timeout=120)
    rec = [json.loads(x) for x in open(os.path.join(lp, "flow", "20160801", "metrics.jsonl"))][-1]
    out["cli_via_service_walls"] = [round(w, 3) for w in walls]
    out["cli_via_service_first_s"] = round(walls[0], 3)
    out["cli_via_service_warm_s"] = round(min(walls[1:] or walls), 3)
    out["via_service_in_process"] = {k: rec.get(k) for k in ("load_s", "day_s", "train_s", "score_s")}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
