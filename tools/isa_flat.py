#!/usr/bin/env python3
"""Per-function FLAT memory instructions (flat_load_* / flat_store_* / flat_atomic_*) and per-kernel resource notes
(VGPR / SGPR spills, private segment) of the gfx950 code objects inside the built library (CPU only: llvm-objdump
on the offload bundles of libfactorysim.so or of the build's objects).

Every device memory access of the env-step is meant to be address-space specific -- ds_* for the arena workspace,
global_* / buffer_* for the records and the arena's global scratch block, s_load / global_load for the scene tables
through the constant address space, scratch_* for private frames.  A FLAT instruction marks a pointer whose
address space the compiler lost (a pointer selected between two address spaces, or a generic pointer parameter of
a non-inlined function) and resolves it per lane at run time; tests/test_build_flags.py asserts there are none.

usage: tools/isa_flat.py [libfactorysim.so | objdir] [--meta]"""
import bisect
import collections
import os
import pathlib
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = pathlib.Path(__file__).resolve().parents[1]


def extract(path):
    """[(label, code object path)] of the gfx950 code objects in a .so / .o (or every .o of a directory), and the
    temporary directory holding them (the caller removes it)"""
    tmp = tempfile.mkdtemp(prefix="isa_flat_")
    src = pathlib.Path(path)
    files = sorted(src.glob("*.o")) if src.is_dir() else [src]
    out = []
    for f in files:
        dst = os.path.join(tmp, f.name)
        shutil.copy(f, dst)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", dst], cwd=tmp, capture_output=True)
        for p in sorted(os.listdir(tmp)):
            if p.startswith(f.name + ".") and "gfx950" in p and os.path.getsize(os.path.join(tmp, p)) > 0:
                out.append((p.replace(".hipv4-amdgcn-amd-amdhsa--gfx950", ""), os.path.join(tmp, p)))
    return out, tmp


def flat_by_function(co_path):
    """{function symbol: Counter(opcode)} of the FLAT instructions, each attributed to its enclosing symbol"""
    sym = subprocess.run([f"{LLVM}/llvm-readelf", "-sW", co_path], capture_output=True, text=True).stdout
    funcs = sorted({(int(p[1], 16), p[7]) for p in (l.split() for l in sym.splitlines())
                    if len(p) >= 8 and p[3] == "FUNC" and p[6] != "UND"})
    addrs = [a for a, _ in funcs]
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co_path], capture_output=True,
                         text=True).stdout
    res = collections.defaultdict(collections.Counter)
    for line in dis.splitlines():
        m = re.match(r"^\s+(flat_\w+).*//\s*([0-9A-Fa-f]+):", line)
        if m:
            i = bisect.bisect_right(addrs, int(m.group(2), 16)) - 1
            res[funcs[i][1] if i >= 0 else "?"][m.group(1)] += 1
    return res


def kernel_meta(co_path):
    """{kernel symbol: {vgpr_count, vgpr_spill_count, sgpr_spill_count, private_segment_fixed_size, ...}} from the
    code object's AMDHSA metadata note"""
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co_path], capture_output=True, text=True).stdout
    out = {}
    for blk in re.split(r"\n\s+- \.", notes):
        m = re.search(r"(?:^|\n)\s*\.?name:\s+(\S+)", blk)
        if not m or m.group(1).endswith(".kd"):
            continue
        d = {}
        for k in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                  "private_segment_fixed_size", "group_segment_fixed_size", "kernarg_segment_size"):
            mm = re.search(r"\.%s:\s+(\d+)" % k, blk)
            if mm:
                d[k] = int(mm.group(1))
        mm = re.search(r"\.uses_dynamic_stack:\s+(\w+)", blk)
        if mm:
            d["uses_dynamic_stack"] = mm.group(1) == "true"
        if d:
            out[m.group(1)] = d
    return out


def demangle(names):
    names = list(names)
    if not names:
        return {}
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
    return dict(zip(names, out.splitlines()))


def scan(path):
    """(flat, meta): {(code object, demangled function): Counter} and {(code object, demangled kernel): notes}"""
    cos, tmp = extract(path)
    flat, meta = {}, {}
    try:
        for label, co in cos:
            f = flat_by_function(co)
            dm = demangle(f)
            for k, c in f.items():
                flat[(label, dm[k])] = c
            m = kernel_meta(co)
            dm = demangle(m)
            for k, v in m.items():
                meta[(label, dm[k])] = v
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return flat, meta


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path = args[0] if args else str(ROOT / "factory_marl_amd" / "libfactorysim.so")
    flat, meta = scan(path)
    for (co, fn), c in sorted(flat.items()):
        print(f"FLAT {co:28s} {sum(c.values()):4d} {fn[:100]}  {dict(c)}")
    if not flat:
        print("no FLAT instructions")
    if "--meta" in sys.argv:
        for (co, k), v in sorted(meta.items()):
            if "step_kernel" in k:
                print(f"META {co:28s} {k[:80]:80s} {v}")


if __name__ == "__main__":
    main()
