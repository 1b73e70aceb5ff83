"""The CPU backend (fm_create(..., device = -1); SURVEY.md §8(b): "A CPU backend (device=-1) exports the same ABI").

No GPU needed: the env-step kernel's own sources (fm_device.hpp) compiled for the host with the 64-lane wave
emulated (fm_simt_host.hpp, fm_cpu.cpp), driven through the same C ABI and FactoryVecEnv.  Checked here against the
oracle on the same inputs, teacher-forced (tests/parity_util.py) and free-running, at the sizes the emulation finishes
in seconds.  Tolerances: fp64 1e-7 relative state error per teacher-forced step (the GPU fp64 gate), fp32 the SURVEY
gate 1e-4 on >= 99% of the steps; integers, RNG and flags bit for bit."""
import os

import numpy as np
import pytest
import torch

import parity_util as pu

A, K = 2, 4


@pytest.fixture(scope="module")
def lib():
    from factory_marl_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libfactorysim.so not built (run `python __graft_entry__.py`)")
    return _lib.load()


def test_emulated_wave_cross_lane_operations(lib):
    """ballot, readlane, DPP row/broadcast moves, ds_bpermute, mbcnt, the 16x16x4 MFMA layout, barriers"""
    assert lib.fm_cpu_selftest() == 0


@pytest.fixture(scope="module")
def trajectory(oracle):
    return pu.rollout(oracle, A, K, 96, seed_actions=11)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_teacher_forced_steps_match_the_oracle(lib, trajectory, precision):
    r = pu.compare(trajectory, precision, A, K, device="cpu")
    s = pu.summary(r)
    assert s["int_bad"] == 0 and s["flag_bad"] == 0, s
    if precision == "fp64":
        assert s["worst"] <= 1e-7, s
        assert s["obs_worst"] <= 1e-6 and s["rew_worst"] <= 1e-6, s
    else:
        assert s["within"] >= 0.99 and s["worst"] <= 1e-3, s
    assert s["max_cubes"] >= 2  # cubes spawned and in contact with the belt over the trajectory


def test_ik_toggle_class_matches_the_oracle(lib, oracle):
    tr = pu.rollout(oracle, A, K, 24, env_class="PauseIKToggleEnv", seed_actions=5)
    r = pu.compare(tr, "fp64", A, K, env_class="PauseIKToggleEnv", device="cpu")
    s = pu.summary(r)
    assert s["int_bad"] == 0 and s["flag_bad"] == 0 and s["worst"] <= 1e-7, s
    assert float(r["ik_err"].max()) <= 1e-7


def test_cpu_handle_refuses_the_gpu_only_entry_points(lib):
    """rendering and the per-phase profile are GPU features: the CPU handle reports an error, never a silent no-op"""
    import ctypes as C

    from factory_marl_amd import _lib

    c = _lib.FmConfig()
    lib.fm_config_default(C.byref(c))
    c.num_arenas = 1
    c.num_arms, c.max_num_objects = A, K
    h = C.c_void_p()
    assert lib.fm_create(C.byref(c), -1, None, C.byref(h)) == 0
    try:
        buf = (C.c_uint64 * 64)()
        assert lib.fm_profile(h, 1, buf) != 0
        assert lib.fm_last_error().decode()
    finally:
        lib.fm_destroy(h)


def test_state_roundtrip_on_the_host(lib):
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    env = FactoryVecEnv(3, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=A, max_num_objects=K, seed=3),
                        device="cpu", precision="fp64")
    env.reset()
    s0 = env.get_state()
    env.set_state(s0)
    assert np.array_equal(env.get_state(), s0)
    assert env.device == torch.device("cpu")
    env.close()


def test_config3_scene_matches_the_oracle(lib, oracle):
    """the (2,8) scene of configs 3 / 4 on the host: teacher-forced fp64 against the oracle"""
    tr = pu.rollout(oracle, 2, 8, 24, seed_actions=3)
    r = pu.compare(tr, "fp64", 2, 8, device="cpu")
    s = pu.summary(r)
    assert s["int_bad"] == 0 and s["flag_bad"] == 0 and s["worst"] <= 1e-7, s


def test_results_do_not_depend_on_the_lane_order(lib, trajectory, tmp_path):
    """the kernel's lanes hand data to each other only at SYNC(): running each emulated wave's lanes
    in reverse order (FACTORYSIM_CPU_REVERSE=1, read once per process: a child process) gives the same env-steps --
    up to the summation order of the LDS float64 atomics (the J'f scatter), so within 1e-9 relative in fp64"""
    import subprocess
    import sys

    recs, acts, _ = trajectory
    np.savez(tmp_path / "in.npz", recs=recs[:24], acts=acts[:24])
    code = f"""
import sys, numpy as np
sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
sys.path.insert(0, {repr(os.path.dirname(os.path.abspath(__file__)))})
import parity_util as pu, torch
d = np.load({repr(str(tmp_path / "in.npz"))})
env = pu.gpu_env(len(d["recs"]), "fp64", {A}, {K}, device="cpu")
env.set_state(d["recs"])
env.step_tensors(torch.as_tensor(d["acts"]))
np.save({repr(str(tmp_path / "out.npy"))}, env.get_state())
"""
    env = dict(os.environ, FACTORYSIM_CPU_REVERSE="1")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=600)
    rev = np.load(tmp_path / "out.npy")
    fwd_env = pu.gpu_env(24, "fp64", A, K, device="cpu")
    fwd_env.set_state(recs[:24])
    fwd_env.step_tensors(torch.as_tensor(acts[:24]))
    fwd = fwd_env.get_state()
    from factory_marl_amd import state as st

    for s in range(24):
        gd, gi, gr = st.unpack(A, K, fwd[s])
        rd, ri, rg = st.unpack(A, K, rev[s])
        assert np.array_equal(gi, ri) and np.array_equal(gr, rg), s
        qd, vd = pu.state_err(A, K, rd, gd)
        assert max(qd.max(), vd.max()) <= 1e-9, (s, qd.max(), vd.max())


def test_crowded_states_through_the_wide_kernel_on_the_host(lib, oracle):
    """(2,4) records whose first stage holds 66-110 contacts (arms pressed into the table, the belt and each other):
    on the host, as on the GPU, the 64-contact kernel abandons them and the float64 wide kernel steps them
    (fm_cpu_fixed.cpp); fp64 against the oracle within 1e-7, integer state / flags exact.  These env-steps also run
    the general register factor (chol_sparse_rl: arms coupled to cubes), whose broadcasts round 6 moved out of a
    lane-dependent branch -- the emulator stops on a cross-lane operation reached by part of the wave"""
    import test_gpu_parity as tg

    traj = tg._crowded_trajectory(oracle)
    r = pu.compare(traj, "fp64", A, K, device="cpu")
    assert not r["flag_bad"] and not r["int_bad"] and not r["reset_bad"], (r["flag_bad"], r["int_bad"], r["reset_bad"])
    assert int(r["counters"][:, 8].sum()) == len(traj[0]) and int(r["counters"][:, 0].sum()) == 0
    assert r["errs"].max() <= 1e-7, r["errs"].max()


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_ik_grasps_on_the_host(lib, oracle, precision):
    """PauseIKToggleEnv over 96 env-steps (the IK base policy grasps cubes: arm-cube contacts couple two trees, the
    non-arrowhead substeps) on the host against the oracle: fp64 within 1e-5; fp32 within the SURVEY gate on >= 99 %
    of the steps and 1e-3 on every step, the nearer of the 1e-12 and the 1e-8 oracle (the IK-class kernel's float64 arm
    poses, FixedDims::f64ik -- with the float arm chain 88.5 % of these steps were within, worst 1.55)"""
    tr = pu.rollout(oracle, A, K, 96, env_class="PauseIKToggleEnv", seed_actions=7)
    alt = pu.restep_at_tolerance(oracle, A, K, tr, 1e-8, "PauseIKToggleEnv") if precision == "fp32" else None
    r = pu.compare(tr, precision, A, K, env_class="PauseIKToggleEnv", device="cpu", alt=alt)
    s = pu.summary(r)
    assert s["int_bad"] == 0 and s["flag_bad"] == 0, s
    if precision == "fp64":
        assert s["worst"] <= 1e-5, s
    else:
        print(s, pu.two_oracle_gate(r, frac=0.99, cap=1e-3))
