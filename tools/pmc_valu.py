#!/usr/bin/env python3
"""VALU work of the env-step kernel per arena env-step from one rocprofv3 --pmc pass (test/measurement infra).

usage: python tools/pmc_valu.py PMC.csv --arenas 4096 --last 3 [--precision fp32] [--out profiles/pmc_valu.json]
Counters (one pass, 8 SQ slots): SQ_INSTS_VALU, SQ_INSTS_VALU_ADD_F32, SQ_INSTS_VALU_MUL_F32, SQ_INSTS_VALU_FMA_F32,
SQ_INSTS_VALU_TRANS_F32, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_WAVES.  Instruction counters count wave-instructions:
lane FLOPs = 64 x (ADD + MUL + TRANS + 2 FMA) -- every lane of the wave, active or not, so an upper bound on the
useful fp32 FLOPs.  Only the last `--last` dispatches of the step-kernel instantiation with the most waves are used (the timed steps after
the pre-roll; SQ_WAVES = the arena count per launch).
"""
import argparse
import csv
import json
from collections import defaultdict


def pass_means(path, last, full=False):
    """mean counters per dispatch over the last `last` dispatches of the step-kernel instantiation with the most waves:
    the (2,4) bench launches the wide rerun kernel after every step (nearly always over an empty list, a few waves) --
    only the main instantiation is the step kernel the line prices (as tools/pmc_traffic.py selects it)"""
    per = defaultdict(dict)
    kname = {}
    for r in csv.DictReader(open(path)):
        if "step_kernel" not in r["Kernel_Name"]:
            continue
        key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
        kname[key] = r["Kernel_Name"]
        per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    waves = defaultdict(list)
    for k, c in per.items():
        waves[kname[k]].append(c.get("SQ_WAVES", 0.0))
    main_k = max(waves, key=lambda n: sorted(waves[n])[len(waves[n]) // 2])
    keys = sorted(k for k in per if kname[k] == main_k)[-last:]
    tot = defaultdict(float)
    for k in keys:
        for c, v in per[k].items():
            tot[c] += v / len(keys)
    return (tot, main_k, keys) if full else tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--arenas", type=int, default=4096)
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--arms", type=int, default=2)
    ap.add_argument("--objects", type=int, default=4)
    ap.add_argument("--out", default="profiles/pmc_valu.json")
    ap.add_argument("--f64", default=None, help="a second pass with SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 + SQ_WAVES: "
                    "the fp32 build's float64 work (master state, narrowphase, Newton iterate) added to the FLOPs")
    a = ap.parse_args()
    tot, main_k, keys = pass_means(a.csv, a.last, full=True)
    if a.f64:
        t64 = pass_means(a.f64, a.last)
        for c, v in t64.items():
            if c.endswith("_F64"):
                tot[c] = v
    n = a.arenas

    def lane_flops(f):
        return 64.0 * (tot.get(f"SQ_INSTS_VALU_ADD_{f}", 0) + tot.get(f"SQ_INSTS_VALU_MUL_{f}", 0) +
                       tot.get(f"SQ_INSTS_VALU_TRANS_{f}", 0) + 2 * tot.get(f"SQ_INSTS_VALU_FMA_{f}", 0))

    f32, f64 = lane_flops("F32"), lane_flops("F64")
    flop = f32 + f64 if a.f64 else (f32 if a.precision == "fp32" else f64)
    rec = {"kernel": main_k, "arenas": n, "precision": a.precision, "A": a.arms, "K": a.objects,
           "dispatches": len(keys), "counters_per_launch": dict(tot),
           "valu_wave_instr_per_arena_step": tot.get("SQ_INSTS_VALU", 0) / n,
           "valu_lane_flops_per_arena_step": flop / n,
           "valu_lane_flops_f32_per_arena_step": f32 / n, "valu_lane_flops_f64_per_arena_step": f64 / n,
           "note": "mean over the last dispatches; lane FLOPs count all 64 lanes of each executed wave-instruction"}
    with open(a.out, "w") as fo:
        json.dump(rec, fo, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
