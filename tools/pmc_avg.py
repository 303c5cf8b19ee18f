#!/usr/bin/env python3
"""Average each counter of rocprofv3 --pmc counter_collection.csv files over dispatches (optionally of kernels
matching a substring): python tools/pmc_avg.py [-k substr] <csv>..."""
import collections
import csv
import sys

args = sys.argv[1:]
pat = ""
if args and args[0] == "-k":
    pat, args = args[1], args[2:]
for f in args:
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f, {k: round(sum(v) / len(v)) for k, v in sorted(acc.items())})
