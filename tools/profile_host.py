#!/usr/bin/env python3
"""Host-side (Python) profile of one pipeline day on the GPU: which host calls dominate a source's
day besides the device work. Usage: python tools/profile_host.py {flow,dns,proxy} [events] [--pcap]"""
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    src = sys.argv[1] if len(sys.argv) > 1 else "proxy"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
    pcap = "--pcap" in sys.argv
    import torch
    from oni355.parallel.comm import init_from_env
    comm = init_from_env("cuda")  # ONI_FORCE_DIST=1: the data-parallel code path on one GPU
    if src == "dns":
        from oni355.synth.dns import generate_dns, write_pcap
        day = generate_dns(n, seed=7)
        from oni355.pipeline.dns import run_dns

        path = None
        if pcap:
            path = os.path.join(tempfile.mkdtemp(), "d.pcap")
            write_pcap(day, path)

        def go():
            cols = day.cols
            if path:
                from oni355.io.decoders import read_pcap_dns
                cols = read_pcap_dns(path)
            return run_dns(cols, K=50, sweeps=200, top_domains=day.top_domains, user_domain="intel", device="cuda")
    elif src == "proxy":
        from oni355.synth.proxy import generate_proxy
        from oni355.pipeline.proxy import run_proxy
        day = generate_proxy(n, seed=7)

        def go():
            return run_proxy(day.cols, K=20, sweeps=200, device="cuda")
    else:
        from oni355.synth.flow import generate_flows
        from oni355.pipeline.flow import run_flow
        day = generate_flows(n, seed=7)

        def go():
            return run_flow(day.cols, K=20, sweeps=200, device=comm.device, comm=comm)
    go()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    res = go()
    torch.cuda.synchronize()
    pr.disable()
    print(f"{src} day: {time.perf_counter() - t:.3f} s; timings {res.timings}")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(int(os.environ.get("PROFILE_LINES", "35")))
    print(s.getvalue())
    return 0


if __name__ == "__main__":
    sys.exit(main())
