#!/usr/bin/env python3
"""Instruction mix per basic block of one kernel in a hipcc -S (device) listing:
python tools/asm_mix.py <file.s> <kernel symbol prefix> [min block size]"""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().split("\n")
pre = sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 40
start = next(i for i, l in enumerate(lines) if l.startswith(pre) and ":" in l)
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\d+_\d+|\S+):", l)
    if m:
        cur = [m.group(1), []]
        blocks.append(cur)
        continue
    t = l.strip()
    if cur is None or not t or t.startswith(";") or t.startswith("."):
        continue
    cur[1].append(t.split()[0])
tot = Counter()
for name, ins in blocks:
    c = Counter()
    for x in ins:
        k = ("mfma" if x.startswith("v_mfma") else "dpp/perm" if "_dpp" in x or "permlane" in x else
             "trans" if re.match(r"v_(exp|rcp|log|sqrt|rsq|sin|cos)_", x) else "valu" if x.startswith("v_") else
             "lds" if x.startswith("ds_") else "wait" if x.startswith("s_waitcnt") else
             "barrier" if x.startswith("s_barrier") else "vmem" if x.startswith(("global_", "buffer_", "scratch_")) else
             "salu" if x.startswith("s_") else "other")
        c[k] += 1
    tot += c
    if len(ins) >= mn:
        print(name, len(ins), dict(c))
print("total", dict(tot))
