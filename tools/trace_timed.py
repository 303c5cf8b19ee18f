#!/usr/bin/env python3
"""Reproduce a bench line's roofline from the rocprofv3 kernel trace of the SAME run.

Usage: python tools/trace_timed.py <rocprof -d dir> <bench line json>

bench.py times K steps; the dominant kernel (the line's roofline.kernel) is launched once per step.
The trace holds every dispatch of that kernel in launch order: the clock ramp, W warmup steps, the K
timed steps, then (C2) the untimed torch fill_ of write_ceiling. The K timed dispatches are the last K
dispatches of the kernel before the first fill kernel that follows them. Prints their mean / min /
median / max duration, the frac they give (algorithmic bytes per launch / mean / peak), the line's own
HIP-event figures beside it, and the all-dispatch rocprof average (the --stats row)."""
import csv
import glob
import json
import os
import sys

import numpy as np


def main():
    d, line_path = sys.argv[1], sys.argv[2]
    line = None
    for l in open(line_path):
        if l.startswith("{"):
            line = json.loads(l)
    if line is None:
        sys.exit("no JSON line in " + line_path)
    K = int(line["steps"])
    roof = line["roofline"]
    tr = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not tr:
        sys.exit("no kernel_trace.csv under " + d)
    rows = list(csv.DictReader(open(tr[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sim = [k for k, r in enumerate(rows) if "sde_simulate_kernel" in r["Kernel_Name"]]
    # the dominant template = the simulator instantiation with the most dispatches
    names = {}
    for k in sim:
        names[rows[k]["Kernel_Name"]] = names.get(rows[k]["Kernel_Name"], 0) + 1
    name = max(names, key=names.get)
    idx = [k for k in sim if rows[k]["Kernel_Name"] == name]
    fills = [k for k, r in enumerate(rows) if "FillFunctor" in r["Kernel_Name"] and k > idx[0]]
    # first fill preceded by >= K dispatches of the kernel
    cut = next((f for f in fills if sum(1 for k in idx if k < f) >= K), None)
    before = [k for k in idx if cut is None or k < cut]
    timed = before[-K:]
    dur = np.array([(int(rows[k]["End_Timestamp"]) - int(rows[k]["Start_Timestamp"])) / 1e6 for k in timed])
    alld = np.array([(int(rows[k]["End_Timestamp"]) - int(rows[k]["Start_Timestamp"])) / 1e6 for k in idx])
    B = float(roof.get("algorithmic_bytes_per_launch") or 0)
    peak = float(roof["peak"])
    out = {
        "kernel": name, "dispatches_total": len(idx), "timed_dispatches": len(timed),
        "rocprof_timed_ms_mean": float(dur.mean()), "rocprof_timed_ms_min": float(dur.min()),
        "rocprof_timed_ms_median": float(np.median(dur)), "rocprof_timed_ms_max": float(dur.max()),
        "rocprof_all_ms_mean": float(alld.mean()),
        "line_kernel_ms": roof["kernel_ms"], "line_kernel_ms_min": roof.get("kernel_ms_min"),
        "line_kernel_ms_median": roof.get("kernel_ms_median"), "line_kernel_ms_max": roof.get("kernel_ms_max"),
        "line_frac": roof["frac"],
    }
    if roof["unit"] == "GB/s" and B:
        out["frac_from_rocprof_timed"] = B / (dur.mean() / 1e3) / 1e9 / peak
        out["frac_from_rocprof_all"] = B / (alld.mean() / 1e3) / 1e9 / peak
        out["line_vs_rocprof_timed"] = roof["frac"] / out["frac_from_rocprof_timed"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
