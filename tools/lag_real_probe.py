#!/usr/bin/env python3
"""Step-by-step probe of a forced-real 1-rank RCCL group with the lagged X01 (diagnostics):
eager sweeps first, then graph-captured ones, printing after each stage."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ONI_FORCE_DIST", "1")
os.environ.setdefault("ONI_COMM_REAL", "1")
os.environ.setdefault("ONI_X01_LAG", "1")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def main() -> int:
    import torch
    from oni355.parallel import comm as pc
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    comm = pc.init_from_env("cuda")
    print("comm", comm.live, comm.real, flush=True)
    day = generate_flows(20_000, seed=3)
    for graph in ("0", "1"):
        os.environ["ONI_NO_GRAPH"] = "1" if graph == "0" else "0"
        for lag_from in ("1000", "3"):
            os.environ["ONI_X01_LAG_FROM"] = lag_from
            print("run graph", graph, "lag_from", lag_from, flush=True)
            res = run_flow(dict(day.cols), K=20, sweeps=12, maxresults=100, device="cuda:0", comm=comm, eval_every=6)
            torch.cuda.synchronize()
            m = res.lda.model
            print("  ok loglik", res.stats["loglik"], "replays", m.timings.get("graph_replays", 0), "lag", m._lag_live,
                  "x01 ms", m.allreduce_ms_per_sweep(), flush=True)
    comm.barrier()
    pc.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
