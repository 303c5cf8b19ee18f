"""Per-kernel duration summary of a rocprofv3 kernel trace dir, big launches only (the 2^21-row chunks):
python tools/kstat_big.py DIR REGEX -> name, calls >= 1/2 of the max duration, their mean (us)."""
import collections
import csv
import glob
import re
import sys

d, rx = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
dur = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if rx.search(r["Kernel_Name"]):
        dur[r["Kernel_Name"].split("(")[0].replace("void pdeinv::", "")].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for k, v in sorted(dur.items(), key=lambda kv: -max(kv[1])):
    big = [x for x in v if x >= 0.5 * max(v)]
    tot += sum(big) / len(big)
    print(f"{k[:70]:72s} {len(big):4d} {sum(big) / len(big):9.1f}us")
print(f"{'sum of big-launch means':72s} {tot:14.1f}us")
