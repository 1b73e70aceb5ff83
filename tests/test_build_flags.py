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


def _isa(name="libfactorysim.so"):
    import importlib.util

    root = pathlib.Path(__file__).resolve().parents[1]
    so = root / "factory_marl_amd" / name
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
         if n.startswith("void fm::step_kernel<float, fm::FixedDims<2, 4, false, false>, false>")]
    assert len(k) == 1, k
    v = k[0][2]
    assert v["vgpr_spill_count"] == 0 and v["private_segment_fixed_size"] == 0, v
    assert v["vgpr_count"] + v.get("agpr_count", 0) <= 256, v


def test_product_kernels_carry_no_experiment_switches():
    """the A/B and test switches live in the experiment build only (libfactorysim_exp.so, -DFM_EXPERIMENTS=1): in the
    kernel sources every switch is read through FM_XF(M), the constant 0 in the product build, and Model has no
    dbg_flags field there -- so the product's step kernels take a smaller parameter block than the experiment build's
    (the switch word is absent from their kernarg)"""
    src = DEVICE.read_text()
    assert "dbg_flags" not in src and "FM_XF(M)" in src
    dev = (DEVICE.parent / "fm_dev.hpp").read_text()
    m = re.search(r"#if FM_EXPERIMENTS\n\s*int dbg_flags;.*?\n#endif", dev)
    assert m, "Model::dbg_flags must be compiled only into the experiment build"
    assert re.search(r"#else\n#define FM_XF\(M\) 0\n", dev)
    _, meta = _scan()
    _, meta_x = _isa("libfactorysim_exp.so")
    name = "void fm::step_kernel<float, fm::FixedDims<2, 4, false, false>, false>"
    k = [v for (co, n), v in meta.items() if n.startswith(name)]
    kx = [v for (co, n), v in meta_x.items() if n.startswith(name)]
    assert len(k) == 1 and len(kx) == 1
    assert k[0]["kernarg_segment_size"] < kx[0]["kernarg_segment_size"], (k[0], kx[0])


def test_product_library_rejects_experiment_switches():
    """a handle of the product library refuses the switches (FM_EINVAL), on the CPU backend (device = -1)"""
    import ctypes as C

    from factory_marl_amd import _lib

    root = pathlib.Path(__file__).resolve().parents[1]
    if not (root / "factory_marl_amd" / "libfactorysim.so").exists():
        import pytest

        pytest.skip("libfactorysim.so not built")
    L = _lib.load()
    cfg = _lib.FmConfig()
    L.fm_config_default(C.byref(cfg))
    cfg.num_arms, cfg.max_num_objects = 2, 4
    h = C.c_void_p()
    seeds = (C.c_uint64 * 1)(42)
    _lib.check(L.fm_create(C.byref(cfg), -1, seeds, C.byref(h)), L)
    try:
        assert L.fm_set_param(h, b"experiment_flags", 512.0) != 0
        assert b"compiled out" in L.fm_last_error()
        assert L.fm_set_param(h, b"experiment_flags", 0.0) == 0
    finally:
        L.fm_destroy(h)


# VGPR spill ceilings of every step-kernel instantiation of the product library (code-object notes, round 6): the
# benchmark kernel has none; the two-waves-per-SIMD kernels of (2,4) fp64 / IK classes and (2,8) / (2,10) AllFullRL
# trade their spills for occupancy (measured: DESIGN.md §4 / §4c; the (2,10) one, 893 spilled at 8 arenas per CU,
# measured faster than an allocation of the same code with 180, profiles/r06r_ab/); the one-wave kernels keep only the few VGPRs the
# non-inlined IK calls save.  A change that spills more than this is a regression to measure before it ships.
SPILL_CEILING = {
    "float, fm::FixedDims<2, 4, false, false>, false": 0,
    "float, fm::FixedDims<2, 4, false, true>, true": 180,
    "double, fm::FixedDims<2, 4, false, false>, false": 120,
    "double, fm::FixedDims<2, 4, false, false>, true": 260,
    "double, fm::FixedDims<2, 4, true, false>, false": 16,
    "double, fm::FixedDims<2, 4, true, false>, true": 28,
    "float, fm::FixedDims<2, 8, false, false>, false": 50,
    "float, fm::FixedDims<2, 8, false, true>, true": 8,
    "double, fm::FixedDims<2, 8, false, false>, false": 130,
    "double, fm::FixedDims<2, 8, false, false>, true": 8,
    "float, fm::FixedDims<2, 10, false, false>, false": 900,
    "float, fm::FixedDims<2, 10, false, true>, true": 8,
    "double, fm::FixedDims<2, 10, false, false>, false": 135,
    "double, fm::FixedDims<2, 10, false, false>, true": 8,
    "float, fm::FixedDims<4, 16, false, false>, false": 0,
    "float, fm::FixedDims<4, 16, false, true>, true": 8,
    "double, fm::FixedDims<4, 16, false, false>, false": 8,
    "double, fm::FixedDims<4, 16, false, false>, true": 8,
}


def test_step_kernel_spills_within_their_ceilings():
    _, meta = _scan()
    seen = {}
    for (co, n), v in meta.items():
        m = re.match(r"void fm::step_kernel<(.*)>\(fm::StepParams", n)
        if m and "FixedDims" in m.group(1):
            seen[m.group(1)] = v["vgpr_spill_count"]
    assert set(seen) == set(SPILL_CEILING), sorted(set(seen) ^ set(SPILL_CEILING))
    over = {k: (v, SPILL_CEILING[k]) for k, v in seen.items() if v > SPILL_CEILING[k]}
    assert not over, over
