"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per kernel matching argv[2]."""
import re
import sys

cur, rec = None, {}
for l in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1)
        rec[cur] = {}
        continue
    for k in ["VGPRs:", "AGPRs:", "ScratchSize [bytes/lane]:", "Occupancy [waves/SIMD]:", "VGPRs Spill:"]:
        if cur and "remark:" in l and l.split("remark:")[-1].strip().startswith(k):
            rec[cur][k.split("[")[0].strip().rstrip(":").replace(" ", "_")] = l.split(k)[-1].split("[")[0].strip()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for k, v in rec.items():
    if re.search(pat, k):
        print(k[:90], " ".join(f"{a}={b}" for a, b in v.items()))
