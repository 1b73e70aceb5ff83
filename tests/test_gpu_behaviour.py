"""Behavioural statistics of the GPU env against the reference's own MuJoCo numbers (tools/behaviour.py).

* The four saved PPO runs (runs/*.zip -> tests/golden/policy_<run>.npz): each run's ep_info_buffer holds the
  Monitor (r, l) of its last 100 training episodes in MuJoCo (tests/golden/runs_fixtures.npz); the same policy
  (SB3 predict, stochastic) drives the GPU env from reset, one episode per arena.
* The IK base policy (FactoryManipulationEnv): report/report.tex:276-295 quotes mean scores (1.65, 1.17) and a mean
  length of 208.8 over 100 sequential episodes for 2 arms (visualisation.py:55-85), (1.18, 1.16) / 119.74 for 4.

The bands: a policy's return and length within a few percent of its training episodes (measured agreement, DESIGN.md
§3); the base policy per bucket and in length within 2.5 combined standard errors of the report."""
import json
import os
import sys
import types

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _have_gpu():
    return torch.cuda.is_available()


# run -> (band on the mean return, band on the mean length), relative to the run's ep_info_buffer means
# (measured, 512 arenas: rk5rxnav r -3.1 % l -1.6 %; r666unuv -3.0 % / -1.8 %; xfwgqibb +2.1 % / -2.7 %; y6lp1j7k
# +13.7 % / +5.5 % -- the toggle runs' 100-episode buffers carry standard errors of 6-9 % of their means)
POLICY_BANDS = {"rk5rxnav": (0.06, 0.05), "r666unuv": (0.06, 0.05), "xfwgqibb": (0.15, 0.10), "y6lp1j7k": (0.25, 0.15)}


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("run", sorted(POLICY_BANDS))
def test_saved_policy_return_and_length_match_training_episodes(run):
    import behaviour

    out = behaviour.policy(types.SimpleNamespace(run=run, arenas=512, precision="fp32", seeds="arena"))
    ref = out["reference_ep_info"]
    br, bl = POLICY_BANDS[run]
    print(json.dumps({k: out[k] for k in ("r", "l", "finished", "reference_ep_info")}))
    assert out["finished"] == 512
    assert abs(out["r"]["mean"] / ref["r"]["mean"] - 1) <= br, (out["r"], ref["r"])
    assert abs(out["l"]["mean"] / ref["l"]["mean"] - 1) <= bl, (out["l"], ref["l"])


def _within(mean, se, ref, ref_se, k=2.5):
    """|mean - ref| within k combined standard errors (ours and the report's 100-episode sample)"""
    return abs(mean - ref) <= k * np.hypot(se, ref_se)


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_ik_base_policy_report_protocol_two_arms():
    """report.tex:276-282 under its own protocol (visualisation.py:55-80): one FactoryManipulationEnv, seed 42,
    sequential episodes with the TaskManager RNG running on (the kernel's auto-reset), length = t; 60 episodes here
    (the GPU steps one arena at ~5 ms per env-step).  Each bucket's mean score and the mean length
    within 2.5 combined standard errors of the report's (1.65, 1.17) / 208.8 -- the report's standard errors are not
    quoted; ours (same protocol, same n) stand in for them.  The oracle under this protocol
    (profiles/r04_base_policy_2arms_oracle.json, tools/base_policy_study.py): (1.56 +- 0.14, 1.35 +- 0.14), 213.1 +-
    10.5, with the per-arm breakdown of the asymmetry (arm 1 plans after arm 0 and ignores its target: fewer grasp
    attempts, most of the timeouts)"""
    import behaviour

    out = behaviour.base(types.SimpleNamespace(A=2, arenas=0, episodes=60, precision="fp32"))
    seq = out["sequential"]
    print(json.dumps(seq))
    assert seq["episodes"] == 60
    s0, s1, ln = seq["scores0"], seq["scores1"], seq["length_t"]
    assert _within(s0["mean"], s0["se"], 1.65, s0["se"]), s0
    assert _within(s1["mean"], s1["se"], 1.17, s1["se"]), s1
    assert _within(ln["mean"], ln["se"], 208.8, ln["se"]), ln


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_ik_base_policy_four_arms_against_the_report():
    """report.tex:289-295 base row (1.18, 1.16) / 119.74, 4 arms: the large-sample estimate (512 arenas of seeds
    42 + i, first episode each; measured (1.05, 0.95) in 109.6) per bucket within 2.5 combined standard errors, the
    report's taken as the oracle's under the report's protocol (profiles/r04_base_policy_4arms_oracle.json: 0.14,
    0.12, 7.8)"""
    import behaviour

    out = behaviour.base(types.SimpleNamespace(A=4, arenas=512, episodes=0, precision="fp32"))
    par = out["parallel"]
    print(json.dumps(par))
    assert par["finished"] == 512
    assert _within(par["scores0"]["mean"], par["scores0"]["se"], 1.18, 0.14), par["scores0"]
    assert _within(par["scores1"]["mean"], par["scores1"]["se"], 1.16, 0.12), par["scores1"]
    assert _within(par["length_t"]["mean"], par["length_t"]["se"], 119.74, 7.8), par["length_t"]
