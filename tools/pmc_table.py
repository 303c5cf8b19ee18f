"""Per-kernel sums of the counters of one or more rocprofv3 --pmc output dirs: python tools/pmc_table.py DIR..."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void pdeinv::", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r.get("Dispatch_Id", ""))
for k, c in agg.items():
    wc = c.get("SQ_WAVE_CYCLES", 0)
    extra = {}
    if wc:
        for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY"):
            if name in c:
                extra[name + "/WAVE_CYCLES"] = round(c[name] / wc, 3)
    if c.get("SQ_BUSY_CYCLES") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        extra["MFMA_BUSY/BUSY"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_BUSY_CYCLES"], 3)
    print(k[:70], len(n[k]), {a: f"{b:.3g}" for a, b in sorted(c.items())}, extra)
