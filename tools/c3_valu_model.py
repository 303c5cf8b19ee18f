#!/usr/bin/env python3
"""C3 VALU issue model vs the SQ counters.

The C3 launch (sde_simulate_kernel<4, GMM, ..., RES = true>: the simulator with the KFP-GMM residual fused) is
VALU-bound, and its FMA-only roofline fraction (bench.py gmm_sim_flops / gmm_residual_flops against 157.3 TFLOP/s)
cannot say how close it is to the VALU floor: the step also issues transcendentals, Philox's v_mad_u64_u32 and
packed moves. This tool prices the step loop instruction by instruction:
  * the static VALU opcode mix of the kernel's steady-state step loop (hipcc -S of sde.hip: the Depth-1 loop of the
    C3 instantiation), per wave-update;
  * the measured issue cost of each opcode in shader cycles per wave64 instruction (tools/valu_rate.hip, s_memtime,
    at C3's 3 waves per SIMD; opcodes it does not list take the cost of their class);
  -> model issue cycles per wave-update;
and compares it with the SQ pass of the same launch (tools/r05_pmc.sh): SQ_ACTIVE_INST_VALU (quad-cycles summed over
waves) x 4 / wave-updates = measured issue cycles per wave-update, SQ_INSTS_VALU / wave-updates = VALU instructions
per wave-update, and the VALU busy share = SQ_ACTIVE_INST_VALU x 4 / (SIMDs x GRBM_GUI_ACTIVE / 8).

    python tools/c3_valu_model.py <sde device .s> <valu_rate.jsonl> <pmc dir with c3_sq1/, c3_sq2/> > profiles/r05_c3_valu.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys

KERNEL = "_ZN6pdeinv19sde_simulate_kernelILi4ELi1ELb0ELi2ELi8ELb0ELi3ELb1ELb0E"
SIMDS = 1024
N, NSTEP = 1 << 22, 100  # C3: particles, steps (n + 1 updates each)


def loop_mix(asm_path):
    lines = open(asm_path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(KERNEL) and l.split()[0].endswith(":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    # the Depth-1 loop: from its header label to the back-branch to it
    hdr = next(i for i, l in enumerate(body) if "Inner Loop Header: Depth=1" in l or "Loop Header: Depth=1" in l)
    label = body[hdr].split(":")[0]
    back = max(i for i, l in enumerate(body) if l.strip().startswith("s_branch") and l.strip().endswith(label))
    mix = collections.Counter()
    for l in body[hdr:back + 1]:
        t = l.strip()
        if t and not t.startswith((";", ".")) and t.split()[0].startswith("v_"):
            mix[t.split()[0].replace("_e32", "").replace("_e64", "")] += 1
    return mix


def cost(op, rates):
    if op in rates:
        return rates[op], op
    for pre, ref in (("v_pk_", "v_pk_fma_f32"), ("v_exp", "v_exp_f32"), ("v_log", "v_log_f32"), ("v_sin", "v_sin_f32"),
                     ("v_cos", "v_sin_f32"), ("v_rcp", "v_rcp_f32"), ("v_rsq", "v_rcp_f32"), ("v_sqrt", "v_sqrt_f32")):
        if op.startswith(pre):
            return rates[ref], ref
    if "_b64" in op or "_u64" in op or "_i64" in op or "_f64" in op:
        return rates["v_mov_b64"], "v_mov_b64"
    return rates["v_fma_f32"], "v_fma_f32"


def sq_pass(pmc_dir):
    vals = collections.defaultdict(list)
    for p in ("c3_sq1", "c3_sq2"):
        for f in glob.glob(os.path.join(pmc_dir, p, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                if "true, false>" not in r["Kernel_Name"] or "<4, 1, false, 2, 8, false, 3, true" not in r["Kernel_Name"]:
                    continue
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            for d in per.values():
                for k, v in d.items():
                    vals[k].append(v)
    return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}  # median over dispatches


def main():
    mix = loop_mix(sys.argv[1])
    rates = {}
    for l in open(sys.argv[2]):
        if l.startswith("{"):
            d = json.loads(l)
            rates[d["op"]] = d["real_cycles"]
    per_op = {}
    model = 0.0
    for op, n in sorted(mix.items(), key=lambda x: -x[1]):
        c, ref = cost(op, rates)
        per_op[op] = {"per_update": n, "cycles_each": round(c, 3), "priced_as": ref}
        model += n * c
    sq = sq_pass(sys.argv[3])
    wave_updates = (N / 64) * (NSTEP + 1)
    meas = sq["SQ_ACTIVE_INST_VALU"] * 4 / wave_updates
    kcyc = sq["GRBM_GUI_ACTIVE"] / 8
    out = {
        "kernel": "sde_simulate_kernel<4, GMM, K=8, RES> (C3 fused simulate + KFP-GMM residual)",
        "wave_updates": wave_updates,
        "static_valu_per_update": sum(mix.values()),
        "sq_valu_insts_per_update": sq["SQ_INSTS_VALU"] / wave_updates,
        "model_issue_cycles_per_update": model,
        "sq_issue_cycles_per_update": meas,
        "model_over_sq": model / meas,
        "sq_valu_busy": sq["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * kcyc),
        "model_valu_busy": model * wave_updates / (SIMDS * kcyc),
        "kernel_cycles_grbm": kcyc,
        "sq_counters_median": sq,
        "rates_real_cycles": rates,
        "mix": per_op,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
