"""Per-residual HBM traffic of the C5 MLP residual from a tools/profile_r02.sh C5 run: the sum over every
MLP-residual dispatch (mlpf::*, mlp_loss, the runtime fills of the first-order boundary chunks) of FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE, divided by
the number of residual launches (mlp_loss dispatches / chunks per residual).
    python tools/c5_traffic.py gpurun_out/prof_r02/C5 [chunks_per_residual=10] [--per-kernel]
With --per-kernel it also prints the bytes per residual of each kernel (fetch x 2 + write, GB), largest first."""
import csv
import glob
import os
import sys

root = sys.argv[1]
chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 10
tot, loss_calls = {}, {}
by_kernel = {}
for counter, sub, scale in (("FETCH_SIZE", "fetch", 2.0), ("WRITE_SIZE", "write", 1.0)):
    s, n = 0.0, 0
    for f in glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            # + the runtime fills of the first-order boundary chunks (g / a / zetabar planes zeroed, r05)
            if row["Counter_Name"] != counter or not ("mlpf::" in k or "mlp_loss" in k or "fillBuffer" in k):
                continue
            s += float(row["Counter_Value"]) * 1024 * scale
            n += "mlp_loss" in k
            name = k.split("(")[0].replace("void ", "").replace("pdeinv::mlpf::", "").replace("pdeinv::", "")
            by_kernel.setdefault(name, [0.0, 0.0])[sub == "write"] += float(row["Counter_Value"]) * 1024 * scale
    tot[counter], loss_calls[counter] = s, n
per = {c: tot[c] / (loss_calls[c] / chunks) for c in tot}
print({"fetch_bytes_per_residual": per["FETCH_SIZE"], "write_bytes_per_residual": per["WRITE_SIZE"],
       "traffic_bytes_per_residual": per["FETCH_SIZE"] + per["WRITE_SIZE"], "residuals": loss_calls})
if "--per-kernel" in sys.argv:
    res = loss_calls["FETCH_SIZE"] / chunks
    for name, (f, w) in sorted(by_kernel.items(), key=lambda x: -(x[1][0] + x[1][1])):
        print("%-60s read %7.2f GB  write %7.2f GB" % (name[:60], f / res / 1e9, w / res / 1e9))
