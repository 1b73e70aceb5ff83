#!/usr/bin/env python3
"""Summary of a rocprofv3 --pmc SQ pass over the bench (wait / issue fractions, LDS bank conflicts), per step-kernel
instantiation (the (2,4) bench runs the 64-contact kernel and, for the arenas above 64 contacts, the wide rerun kernel);
the headline is the instantiation with the most wave cycles.  usage: python tools/pmc_sq.py counter_collection.csv out.json"""
import csv
import json
import sys
from collections import defaultdict


def fractions(c):
    def div(a, b):
        return c[a] / c[b] if c.get(a) is not None and c.get(b) else None

    return {"wait_any_frac_of_wave_cycles": div("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
            "wait_inst_any_frac": div("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
            "active_inst_frac": div("SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"),
            "lds_bank_conflict_frac_of_lds_active": div("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
            "lds_bank_conflict_frac_of_wave_cycles": div("SQ_LDS_BANK_CONFLICT", "SQ_WAVE_CYCLES"),
            "valu_per_lds": div("SQ_INSTS_VALU", "SQ_INSTS_LDS"),
            # the instruction-cache pass (gpu_measure.sh pmcic): the kernel's ~60k instructions against 64 KB of
            # instruction cache per pair of CUs
            "icache_hit_frac": div("SQC_ICACHE_HITS", "SQC_ICACHE_REQ"),
            "icache_miss_frac": div("SQC_ICACHE_MISSES", "SQC_ICACHE_REQ"),
            "icache_misses_per_wave_kcycle": (1000.0 * c["SQC_ICACHE_MISSES"] / c["SQ_WAVE_CYCLES"]
                                              if c.get("SQ_WAVE_CYCLES") and "SQC_ICACHE_MISSES" in c else None)}


def main(src, dst):
    per = defaultdict(lambda: defaultdict(float))  # counters of a kernel that collected nothing stay 0
    for r in csv.DictReader(open(src)):
        if "step_kernel" in r["Kernel_Name"]:
            per[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    main_k = max(per, key=lambda k: per[k]["SQ_WAVE_CYCLES"])
    c = dict(per[main_k])
    out = {"kernel": main_k, "source": "rocprofv3 --pmc, summed over the bench launches", "counters": c}
    out.update(fractions(c))
    out["by_kernel"] = {k: dict(fractions(v), wave_cycles_share=v["SQ_WAVE_CYCLES"] /
                                sum(x["SQ_WAVE_CYCLES"] for x in per.values())) for k, v in per.items()}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("counters", "by_kernel")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
