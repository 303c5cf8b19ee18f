#!/usr/bin/env python3
"""C3 VALU issue model vs the SQ counters.

The C3 launch (sde_simulate_kernel<4, GMM, ..., RES = true>: the simulator with the KFP-GMM residual fused) is
VALU-bound, and its FMA-only roofline fraction (bench.py gmm_sim_flops / gmm_residual_flops against 157.3 TFLOP/s)
cannot say how close it is to the VALU floor: the step also issues transcendentals, Philox's v_mad_u64_u32 and
packed moves. This tool prices the step loop instruction by instruction:
  * the static VALU opcode mix of the kernel's steady-state step loop (hipcc -S of sde.hip: the Depth-1 loop of the
    C3 instantiation), per wave-update;
  * the SIMD cycles each opcode costs when it saturates the VALU (tools/valu_rate.hip: one opcode per dispatch, 3 waves
    per SIMD = C3's occupancy, 64 independent instructions per loop branch), measured by the SQ itself:
    cpi = kernel cycles (GRBM_GUI_ACTIVE / 8) x SIMDs / SQ_INSTS_VALU (tools/r05_valu_pmc.sh; opcodes it does not
    list take the cost of their class; tools/r05_valu_sweep.sh repeats it at 1, 2, 4, 6 and 8 waves per SIMD);
  -> model: the SIMD cycles per wave-update the loop's VALU needs on its own;
and compares it with the C3 launch's own cycles per wave-update per SIMD (its SQ pass, tools/r05_pmc.sh:
GRBM_GUI_ACTIVE / 8 x SIMDs / wave-updates): their ratio is the VALU issue fraction of the launch. The SQ's
SQ_ACTIVE_INST_VALU is reported beside it but is not an issue-cycle count: it charges one quad-cycle per VALU
instruction (two for a transcendental) whatever the opcode's real cost (0.68-1.26 "busy" in the saturated
microbenchmarks).

    python tools/c3_valu_model.py <sde device .s> <pmc dir: valu_rate/, c3_sq1/, c3_sq2/> > profiles/c3_valu_issue.json
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
                per[r["Dispatch_Id"]]["_dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            for d in per.values():
                for k, v in d.items():
                    vals[k].append(v)
    return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}  # median over dispatches


OPS = {"k_fma": "v_fma_f32", "k_add": "v_add_f32", "k_mul": "v_mul_f32", "k_max": "v_max_f32", "k_mov": "v_mov_b32",
       "k_bitop3": "v_bitop3_b32", "k_and_or": "v_and_or_b32", "k_exp": "v_exp_f32", "k_log": "v_log_f32",
       "k_sin": "v_sin_f32", "k_rcp": "v_rcp_f32", "k_sqrt": "v_sqrt_f32", "k_pk_fma": "v_pk_fma_f32",
       "k_pk_mul": "v_pk_mul_f32", "k_pk_add": "v_pk_add_f32", "k_mov_b64": "v_mov_b64",
       "k_lshl_add_u64": "v_lshl_add_u64", "k_mad_u64": "v_mad_u64_u32", "k_mix_exp_pk": "mix_exp_7pk"}


def calibrate(pmc_dir, sub="valu_rate"):
    """SIMD cycles per instruction of each opcode (median over its dispatches): kernel cycles x SIMDs / VALU insts."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for f in glob.glob(os.path.join(pmc_dir, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].split()[-1]
    cpi = collections.defaultdict(list)
    for d, v in per.items():
        op = OPS.get(name[d])
        if op:
            cpi[op].append(SIMDS * v["GRBM_GUI_ACTIVE"] / 8 / v["SQ_INSTS_VALU"])
    return {op: sorted(v)[len(v) // 2] for op, v in cpi.items()}


def main():
    mix = loop_mix(sys.argv[1])
    rates = calibrate(sys.argv[2])
    per_op = {}
    model = 0.0
    for op, n in sorted(mix.items(), key=lambda x: -x[1]):
        c, ref = cost(op, rates)
        per_op[op] = {"per_update": n, "cycles_each": round(c, 3), "priced_as": ref}
        model += n * c
    # the same mix priced at other occupancies (tools/r05_valu_sweep.sh): a lone opcode stream issues faster with
    # more waves per SIMD, so the W = 8 costs approach the pipe's own issue cost
    by_w = {}
    for sub in sorted(d for d in glob.glob(os.path.join(sys.argv[2], "valu_rate_w*")) if os.path.isdir(d)):
        w = int(sub.rsplit("_w", 1)[1])
        rw = calibrate(sys.argv[2], os.path.basename(sub))
        if "v_fma_f32" in rw and "v_pk_fma_f32" in rw and "v_mov_b64" in rw:
            by_w[w] = sum(n * cost(op, rw)[0] for op, n in mix.items())
    sq = sq_pass(sys.argv[2])
    wave_updates = (N / 64) * (NSTEP + 1)
    meas = sq["SQ_ACTIVE_INST_VALU"] * 4 / wave_updates
    kcyc = sq["GRBM_GUI_ACTIVE"] / 8
    out = {
        "kernel": "sde_simulate_kernel<4, GMM, K=8, RES> (C3 fused simulate + KFP-GMM residual)",
        "wave_updates": wave_updates,
        "static_valu_per_update": sum(mix.values()),
        "sq_valu_insts_per_update": sq["SQ_INSTS_VALU"] / wave_updates,
        "model_issue_cycles_per_update": model,
        "launch_cycles_per_update": SIMDS * kcyc / wave_updates,
        "model_valu_busy": model * wave_updates / (SIMDS * kcyc),
        "model_issue_cycles_per_update_by_waves_per_simd": by_w,
        "model_issue_cycles_per_update_asymptotic": by_w[max(by_w)] if by_w else None,
        "model_valu_busy_asymptotic": by_w[max(by_w)] * wave_updates / (SIMDS * kcyc) if by_w else None,
        "model_valu_busy_by_waves_per_simd": {w: c * wave_updates / (SIMDS * kcyc) for w, c in by_w.items()},
        "sq_active_inst_valu_cycles_per_update": meas,
        "sq_active_inst_valu_share": sq["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * kcyc),
        "kernel_cycles_grbm": kcyc,
        "profiled_kernel_ms": sq["_dur_ns"] / 1e6,
        "profiled_clock_ghz": kcyc / sq["_dur_ns"],
        "sq_counters_median": sq,
        "cpi_simd_cycles": rates,
        "mix": per_op,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
