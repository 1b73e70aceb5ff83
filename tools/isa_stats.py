#!/usr/bin/env python3
"""Per-kernel resource summary of a --save-temps gfx950 .s file: VGPR/AGPR/SGPR, spills, LDS, instruction
counts (total, LDS, VALU, s_waitcnt).  Used to compare kernel variants without a GPU."""
import re
import sys


def stats(path):
    txt = open(path).read()
    out = {}
    # function bodies
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\.Lfunc_end", txt, re.S | re.M):
        name, body = m.group(1), m.group(2)
        ins = [l.strip() for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((";", "."))]
        out[name] = dict(instr=len(ins), ds=sum(i.startswith("ds_") for i in ins),
                         valu=sum(i.startswith("v_") for i in ins),
                         waitcnt=sum(i.startswith("s_waitcnt") for i in ins),
                         readlane=sum(i.startswith("v_readlane") for i in ins))
    for m in re.finditer(r"\.name:\s+(_Z\w+)\n(.*?)(?=\n  - \.|\Z)", txt, re.S):
        pass
    meta = re.findall(r"\.agpr_count:\s+(\d+).*?\.name:\s+(\S+).*?\.sgpr_spill_count:\s+(\d+).*?\.vgpr_count:\s+(\d+)"
                      r".*?\.vgpr_spill_count:\s+(\d+)", txt, re.S)
    for agpr, name, sspill, vgpr, vspill in meta:
        out.setdefault(name, {}).update(agpr=int(agpr), vgpr=int(vgpr), sgpr_spill=int(sspill), vgpr_spill=int(vspill))
    return out


if __name__ == "__main__":
    for k, v in stats(sys.argv[1]).items():
        if "step_kernel" in k or len(sys.argv) > 2:
            print(k[:60], v)
