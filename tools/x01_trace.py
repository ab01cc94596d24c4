#!/usr/bin/env python3
"""Per-sweep X01 anatomy from a rocprofv3 kernel trace of a forced-real day (ONI_FORCE_DIST=1
ONI_COMM_REAL=1): the RCCL kernel between each sweep's count pass and its k_apply, with the pack /
unpack around it, and the gaps. Shows the collective was replayed inside the sweep graphs (one per
sweep, in stream order with the sampler kernels).

  python tools/x01_trace.py gpurun_out/<tag>/prof_N/run_kernel_trace.csv > summary.json
"""
import csv
import json
import statistics
import sys


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)", "").split("(")[0]
    for key in ("k_gibbs_x1", "k_gibbs_ldsg", "k_gibbs_mh", "k_gibbs", "k_wdelta_recount", "k_recount", "k_x01_pack",
                "k_x01_unpack", "rcclGenericKernel", "k_apply", "copyBuffer", "elementwise_kernel"):
        if key in n:
            return key
    return n[-40:]


def main(path: str) -> int:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    sweeps = []
    for i, (k, t0, t1) in enumerate(seq):
        if not k.startswith("k_gibbs"):
            continue
        # the sweep: sampler ... up to its k_apply
        j = i + 1
        parts = {k: t1 - t0}
        order = [k]
        while j < len(seq) and seq[j][0] != "k_apply" and not seq[j][0].startswith("k_gibbs"):
            parts[seq[j][0]] = parts.get(seq[j][0], 0) + seq[j][2] - seq[j][1]
            order.append(seq[j][0])
            j += 1
        if j < len(seq) and seq[j][0] == "k_apply":
            order.append("k_apply")
            parts["k_apply"] = seq[j][2] - seq[j][1]
            parts["sweep_span"] = seq[j][2] - t0
            x = [s for s in seq[i + 1:j] if s[0] in ("k_x01_pack", "rcclGenericKernel", "k_x01_unpack")]
            if x:
                parts["x01_span"] = x[-1][2] - x[0][1]
            sweeps.append((tuple(order), parts))
    with_rccl = [p for o, p in sweeps if "rcclGenericKernel" in o]
    out = {"trace": path, "sweeps_found": len(sweeps), "sweeps_with_rccl_kernel": len(with_rccl),
           "kernel_order_most_common": list(__import__("collections").Counter(
               o for o, p in sweeps if "rcclGenericKernel" in o).most_common(1)[0][0]) if with_rccl else [],
           "median_us": {k: round(statistics.median(p[k] for p in with_rccl if k in p) / 1e3, 2)
                         for k in sorted({k for p in with_rccl for k in p})} if with_rccl else {}}
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
