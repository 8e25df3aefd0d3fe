"""Summarise scripts/pmc_valu.sh output: per eval-kernel dispatch averages and a VALU roofline.

FP64 VALU peak (MI355X): 78.6 TFLOP/s = 256 CUs x 4 SIMDs x 16 FMA lanes x 2 x 2.4 GHz, i.e. one
wave64 FP64 instruction per SIMD per 4 cycles; other VALU (f32 / int) one per 2 cycles.
usage: python scripts/valu_report.py gpurun_out/pmc_valu/<config>
"""
import csv
import glob
import json
import os
import sys

CLK = 2.4e9
SIMDS = 256 * 4
FP64_PEAK = 78.6e12


def counters(d):
    per = {}
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if "cpl_eval" not in row["Kernel_Name"]:
                continue
            per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
            per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in per.items()}


def kernel_ns(d):
    for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
        for row in csv.DictReader(open(f)):
            if "cpl_eval" in row["Name"]:
                return float(row["AverageNs"]), row["Name"]
    return None, None


def report(d):
    c = counters(d)
    ns, name = kernel_ns(d)
    t = ns * 1e-9
    f64 = c.get("SQ_INSTS_VALU_ADD_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) + c.get("SQ_INSTS_VALU_FMA_F64", 0) \
        + c.get("SQ_INSTS_VALU_TRANS_F64", 0)
    valu = c["SQ_INSTS_VALU"]
    issue_cycles = 4 * f64 + 2 * (valu - f64)          # per-SIMD issue cycles, summed over waves
    t_valu = issue_cycles / (SIMDS * CLK)
    flops = c.get("SQ_INSTS_VALU_FLOPS_FP64", 0) + c.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0)
    return {
        "kernel": name, "kernel_us": ns / 1e3, "counters_per_dispatch": c,
        "valu_insts": valu, "fp64_insts": f64, "fp64_share": f64 / valu,
        "valu_issue_bound_us": t_valu * 1e6, "valu_issue_frac": t_valu / t,
        "fp64_tflops": flops / t / 1e12, "fp64_frac_of_peak": flops / t / FP64_PEAK,
        "wait_any_frac": c.get("SQ_WAIT_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1),
        "active_valu_frac_of_wave_cycles": c.get("SQ_ACTIVE_INST_VALU", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1),
    }


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(json.dumps({"dir": d, **report(d)}))
