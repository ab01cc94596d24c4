import sys, time, os, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
from oni355.synth.dns import generate_dns, write_pcap
from oni355.io.decoders import read_pcap_dns
day = generate_dns(2_000_000, seed=7)
p = "/tmp/d.pcap"
t = time.perf_counter(); write_pcap(day, p); tw = time.perf_counter() - t
out = {"pcap_MB": os.path.getsize(p) / 1e6, "write_s": tw, "cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
for th in (0, 1, 4, 8, 16):
    ts = []
    for _ in range(3):
        t = time.perf_counter(); c = read_pcap_dns(p, threads=th); ts.append(time.perf_counter() - t)
    out[f"decode_s_threads{th}"] = round(min(ts), 4)
print(json.dumps(out))
