#!/usr/bin/env python3
"""Summary of a rocprofv3 --pmc SQ pass over the bench (wait / issue fractions, LDS bank conflicts) for the step
kernel.  usage: python tools/pmc_sq.py counter_collection.csv out.json"""
import csv
import json
import sys
from collections import defaultdict


def main(src, dst):
    tot = defaultdict(float)
    name = None
    for r in csv.DictReader(open(src)):
        if "step_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            name = r["Kernel_Name"]
    c = dict(tot)
    out = {"kernel": name, "source": "rocprofv3 --pmc, summed over the bench launches", "counters": c,
           "wait_any_frac_of_wave_cycles": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
           "wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
           "active_inst_frac": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"],
           "lds_bank_conflict_frac_of_lds_active": c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"],
           "valu_per_lds": c["SQ_INSTS_VALU"] / c["SQ_INSTS_LDS"]}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters"}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
