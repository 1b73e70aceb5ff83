"""Build-recipe guards for factory_marl_amd/csrc/Makefile (CPU only).

The scene kernels are built as one object per (scene, precision) so each precision gets its own flags: the
fp32 objects add -fno-slp-vectorize (+4.6 % env-steps/s).  Round 1 kept that flag off the fp64
objects after their parity failed with it; round 2 traced the failure to the compiler-only SYNC() (no wave
barrier, no fences) and, with SYNC() a real wave barrier, both flag sets pass the fp64 parity sweep
identically (gpurun_out/r02a, profiles/r02_parity.md).  These checks keep the per-precision split.
"""
import pathlib
import re

MAKEFILE = pathlib.Path(__file__).resolve().parents[1] / "factory_marl_amd" / "csrc" / "Makefile"
DEVICE = pathlib.Path(__file__).resolve().parents[1] / "factory_marl_amd" / "csrc" / "fm_device.hpp"


def _rules():
    text = MAKEFILE.read_text()
    rules = {}
    for m in re.finditer(r"^(\$\(OBJDIR\)/fm_fixed_%_f(32|64)\.o):.*\n\t(.*)$", text, re.M):
        rules[m.group(2)] = m.group(3)
    return text, rules


def test_fixed_objects_split_by_precision():
    _, rules = _rules()
    assert set(rules) == {"32", "64"}
    assert "-DFM_PREC=32" in rules["32"] and "-DFM_PREC=64" in rules["64"]


def test_slp_flag_on_fp32_objects():
    text, rules = _rules()
    hipflags = re.search(r"^HIPFLAGS \?=(.*(?:\\\n.*)*)", text, re.M).group(1)
    assert "-fno-slp-vectorize" not in hipflags
    assert "$(F32FLAGS)" in rules["32"]
    assert "$(F64FLAGS)" in rules["64"]


def test_sync_is_a_wave_barrier_with_fences():
    """the lanes of an arena hand data to each other through LDS: SYNC() must be a wave barrier plus
    wavefront-scope release/acquire fences, not a compiler-only memory clobber"""
    src = DEVICE.read_text()
    m = re.search(r"#define SYNC\(\)(.*?)while \(0\)", src, re.S)
    assert m, "SYNC() macro not found"
    body = m.group(1)
    assert "__builtin_amdgcn_wave_barrier" in body
    assert "__ATOMIC_RELEASE" in body and "__ATOMIC_ACQUIRE" in body and '"wavefront"' in body


def _isa():
    import importlib.util

    root = pathlib.Path(__file__).resolve().parents[1]
    so = root / "factory_marl_amd" / "libfactorysim.so"
    if not so.exists() or not pathlib.Path("/opt/rocm/lib/llvm/bin/llvm-objdump").exists():
        import pytest

        pytest.skip("libfactorysim.so not built (python -c 'import __graft_entry__ as g; g.build()') or no ROCm llvm")
    spec = importlib.util.spec_from_file_location("isa_flat", root / "tools" / "isa_flat.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.scan(str(so))


_SCAN = {}


def _scan():
    if "r" not in _SCAN:
        _SCAN["r"] = _isa()
    return _SCAN["r"]


def test_no_flat_instructions_in_the_library():
    """every device function of libfactorysim.so (step / reset / debug kernels and the non-inlined IK functions)
    accesses memory through address-space-specific instructions: no flat_load / flat_store / flat_atomic.  A FLAT
    access is a pointer whose address space the compiler lost (a pointer selected between LDS and global or
    kernarg memory, a generic parameter of a non-inlined function); round 4's aperture-violation fault came from the
    one kernel family that carried them"""
    flat, _ = _scan()
    bad = {f"{co}: {fn[:90]}": dict(c) for (co, fn), c in flat.items()}
    assert not bad, bad


def test_step_kernels_have_a_fixed_private_segment():
    """no step kernel needs a dynamic stack (the private segment the runtime allocates is the one the code object
    declares)"""
    _, meta = _scan()
    ks = {k: v for k, v in meta.items() if "step_kernel" in k[1]}
    assert ks
    assert not [k for k, v in ks.items() if v.get("uses_dynamic_stack")], ks


def test_benchmark_kernel_does_not_spill():
    """the config-2 kernel (step_kernel<float, FixedDims<2, 4>, AllFullRL>) is register-allocated for two waves per
    SIMD (256 registers per lane) without VGPR spills and without a private segment: round 4 spilled 180 VGPRs
    (660 B of scratch per lane, ~20 GB of memory-fabric traffic per launch); hoisted lane- and arena-derived values
    were the spill set (fm_device.hpp lane_id / opaque_uniform)"""
    _, meta = _scan()
    k = [(co, n, v) for (co, n), v in meta.items()
         if n.startswith("void fm::step_kernel<float, fm::FixedDims<2, 4, false>, false>")]
    assert len(k) == 1, k
    v = k[0][2]
    assert v["vgpr_spill_count"] == 0 and v["private_segment_fixed_size"] == 0, v
    assert v["vgpr_count"] + v.get("agpr_count", 0) <= 256, v
