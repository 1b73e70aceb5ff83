"""Build-recipe guards for factory_marl_amd/csrc/Makefile (CPU only).

The fp32 scene kernels are built with -fno-slp-vectorize (faster); the same flag on the fully unrolled fp64
fixed-scene kernel miscompiles silently (the fp64 teacher-forced parity tests fail by orders of magnitude), so the
fp64 objects must keep the default flags.  These checks catch a recipe edit that would reintroduce that.
"""
import pathlib
import re

MAKEFILE = pathlib.Path(__file__).resolve().parents[1] / "factory_marl_amd" / "csrc" / "Makefile"


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


def test_slp_flag_only_on_fp32_objects():
    text, rules = _rules()
    hipflags = re.search(r"^HIPFLAGS \?=(.*(?:\\\n.*)*)", text, re.M).group(1)
    assert "-fno-slp-vectorize" not in hipflags
    assert "$(F32FLAGS)" in rules["32"]
    assert "$(F32FLAGS)" not in rules["64"] and "slp" not in rules["64"]
    assert re.search(r"^F64FLAGS \?=\s*$", text, re.M), "fp64 objects must build with the default flags"
