"""Summarise a tools/profile_r02.sh run: per config, per kernel name, the median FETCH_SIZE (x2, the gfx950
correction of MI355X_MICROARCH.md) and WRITE_SIZE bytes per dispatch, and the kernel-trace averages.
    python tools/pmc_summary.py gpurun_out/prof_r02 > profiles/r02_pmc_summary.json"""
import csv
import glob
import json
import os
import statistics
import sys

root = sys.argv[1]
out = {}
for cdir in sorted(glob.glob(os.path.join(root, "C*"))):
    C = os.path.basename(cdir)
    rec = {"kernels": {}}
    for counter, sub, scale in (("FETCH_SIZE", "fetch", 2.0), ("WRITE_SIZE", "write", 1.0)):
        for f in glob.glob(os.path.join(cdir, sub, "**", "*counter_collection.csv"), recursive=True):
            vals = {}
            for row in csv.DictReader(open(f)):
                if row["Counter_Name"] != counter:
                    continue
                vals.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]) * 1024 * scale)
            for k, v in vals.items():
                d = rec["kernels"].setdefault(k[:160], {})
                d[counter.lower() + "_bytes_median"] = statistics.median(v)
                d[counter.lower() + "_dispatches"] = len(v)
    for f in glob.glob(os.path.join(cdir, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            d = rec["kernels"].get(row["Name"][:160])
            if d is not None:
                d["trace_avg_ns"] = float(row["AverageNs"])
                d["trace_calls"] = int(row["Calls"])
    try:
        rec["bench"] = json.loads([l for l in open(os.path.join(cdir, "bench.json")) if l.startswith("{")][0])
    except Exception:
        pass
    out[C] = rec
print(json.dumps(out, indent=1))
