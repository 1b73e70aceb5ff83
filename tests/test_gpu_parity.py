"""GPU parity: the HIP env-step (libfactorysim.so through its C ABI) against the oracle.

Teacher forcing: the oracle runs an episode with random AllFullRL actions; its full arena state after
each env-step (physics stage + task layer, exported in the product's record layout) is loaded into one
GPU arena each, every arena is stepped once with the action the oracle used, and the GPU's resulting
state / obs / reward / flags are compared with the oracle's next step.
Tolerances: SURVEY.md §8(d) -- |dq| <= 1e-4 * max(|ref|, 1), |dv| <= 1e-4 * max(|ref|, 0.1); integer
task state, scores, num_obj, done / out_of_reach / force flags bit-exact.  The fp64 build is also held
to 1e-7 (same algorithm, same precision as the oracle).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import parity_util as pu  # noqa: E402

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

A, K = 2, 4


def _have_gpu():
    return torch.cuda.is_available()


def _rollout(oracle, A_, K_, T, reward="progress", seed_actions=7):
    return pu.rollout(oracle, A_, K_, T, reward=reward, seed_actions=seed_actions)


@pytest.fixture(scope="module")
def trajectory(oracle):
    return _rollout(oracle, A, K, 96)


def _gpu_env(n, precision, A_=A, K_=K, env_class="AllFullRLProgressRewardEnv"):
    return pu.gpu_env(n, precision, A_, K_, env_class)


def _compare(trajectory, precision, tol_rel, A_=A, K_=K, env_class="AllFullRLProgressRewardEnv"):
    r = pu.compare(trajectory, precision, A_, K_, env_class, verbose_tol=10 * tol_rel)
    r["tol"] = tol_rel
    return r


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_reset_obs_matches_oracle(oracle):
    for prec in ["fp64", "fp32"]:
        env = _gpu_env(4, prec)
        obs = env.obs.cpu().numpy()
        e = oracle.Env(A, K, 42)
        ref = e.reset()
        for i in range(4):
            np.testing.assert_array_equal(obs[i], ref)
        env.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_teacher_forced_fp64(trajectory):
    r = _compare(trajectory, "fp64", 1e-7)
    print(f"fp64 teacher-forced: worst rel err {r['errs'].max():.3e}, obs {r['obs_err'].max():.2e}, "
          f"reward {r['rew_err'].max():.2e}; counters {r['counters'].sum(0)}")
    assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
    assert r["errs"].max() <= 1e-7
    assert r["obs_err"].max() <= 1e-5 and r["rew_err"].max() <= 1e-6
    assert r["counters"][:, 0].sum() == 0  # no contacts dropped for capacity


@pytest.fixture(scope="module")
def long_trajectory(oracle):
    """300 env-steps from reset: every cube of the (2, 4) scene spawned, landed, scored or dropped, a force
    termination and its auto-reset (seed 21)"""
    return _rollout(oracle, A, K, 300, seed_actions=21)


@pytest.fixture(scope="module")
def long_trajectory_tol8(oracle, long_trajectory):
    """the long trajectory's states and actions stepped by the oracle at MuJoCo's 1e-8 Newton tolerance"""
    return pu.restep_at_tolerance(oracle, A, K, long_trajectory, 1e-8)


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("which", ["short", "long"])
def test_teacher_forced_fp32(trajectory, long_trajectory, long_trajectory_tol8, which):
    r = pu.compare(trajectory if which == "short" else long_trajectory, "fp32", A, K, verbose_tol=1e-3,
                   alt=None if which == "short" else long_trajectory_tol8)
    e = r["errs"]
    frac = float(np.mean(e <= 1e-4))
    print(f"fp32 teacher-forced (SURVEY tolerance 1e-4 rel): {frac:.1%} of {len(e)} steps within; "
          f"median {np.median(e):.2e}, worst {e.max():.2e}; integer/flag divergences "
          f"{len(r['int_bad'])}/{len(r['flag_bad'])}; obs worst {r['obs_err'].max():.2e}; "
          f"missing steps {list(r['err_steps'][e > 1e-4])}")
    assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
    assert not r["reset_bad"] and (r["resets"] == 0 or r["reset_err"].max() <= 1e-4), (r["reset_bad"], r["reset_err"])
    # fp32 physics over a float64 master state in a z-shifted frame, contact geometry (narrowphase) and the Newton
    # iterate in float64, MuJoCo's 1e-8 Newton tolerance: measured 98.96 % (96 steps: one miss, the
    # first landing impact at step 6, 2.3e-4) and 99.33 % (300 steps: the landing and step 166, where a cube spinning
    # at 8.8 rad/s is struck -- a chaotic contact event, 0.13; the fp64 build matches it to 1e-10)
    if which == "short":
        assert frac >= 0.985 and e.max() <= 5e-4, (frac, e.max())
    else:
        # round 4 (contact points relative to their cube, profiles/r04_parity.md): 296 of 299 steps -- the first
        # landing (step 6, 3.4e-4), a cube spinning at 3.8 rad/s (step 112, 1.05e-4) and step 166 (0.133, a struck
        # spinning cube, missed the same way by the float64 oracle at MuJoCo's 1e-8 tolerance).  Step 166 is a
        # bifurcation on which the 1e-12 and the 1e-8 oracle part: the per-step gate takes the nearer of the two --
        # within 1e-4 on >= 99 % of the steps and <= 1e-3 on every step (no cap of 0.15 on any step)
        assert frac >= 0.989, (frac, np.sort(e)[-3:])
        within, worst, missing = pu.two_oracle_gate(r, frac=0.99, cap=1e-3)
        print(f"  nearer of the 1e-12 / 1e-8 oracles: {within:.2%} within 1e-4, worst {worst:.2e}, missing {missing}")
    assert np.median(e) <= 1e-5
    # the same algorithm in plain single precision (liboracle_f32.so, tools/fp32_floor.py --float-oracle) on the
    # same trajectory: the kernel (float64 master state, z-shifted frame) must hold the gate at least as often,
    # and on the 96-step trajectory every step the kernel misses is one the float restatement misses too
    ff = _float_floor(*((A, K, 96, 7) if which == "short" else (A, K, 300, 21)))
    print(f"float restatement: {ff['within']:.1%} within, missing {ff['missing_steps'][:16]}")
    assert frac >= ff["within"]
    if which == "short":
        assert set(r["err_steps"][e > 1e-4]) <= set(ff["missing_steps"])


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_fp32_against_mujoco_tolerance_oracle(oracle):
    """the fp32 build (MuJoCo's 1e-8 Newton tolerance) against the oracle stepped at that same tolerance from the
    same states: the SURVEY gate on >= 99 % of the long trajectories' env-steps with the worst step under 5e-4
    (round 4: 99.67 / 99.67 / 99.6 %, worst 1.05e-4 / 3.1e-4 / 1.6e-4).  Against the 1e-12 oracle the same kernel
    misses a few more steps (test_teacher_forced_fp32) -- exactly the steps the float64 oracle itself misses at
    1e-8 (tools/tolerance_floor.py): those are MuJoCo's tolerance, not fp32 arithmetic"""
    for A_, K_, T, seed in [(2, 4, 300, 21), (2, 8, 300, 5), (2, 10, 250, 9)]:
        traj = pu.restep_at_tolerance(oracle, A_, K_, _rollout(oracle, A_, K_, T, seed_actions=seed), 1e-8)
        r = _compare(traj, "fp32", 1e-4, A_, K_)
        e = r["errs"]
        frac = float(np.mean(e <= 1e-4))
        print(f"fp32 ({A_},{K_})x{T} vs the 1e-8 oracle: {frac:.2%} within 1e-4, worst {e.max():.2e}")
        assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
        assert frac >= 0.99 and e.max() <= 5e-4, (frac, e.max())


def _float_floor(A_, K_, T, seed):
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import fp32_floor

    return fp32_floor.summarize(fp32_floor.float_oracle_study(A_, K_, T, seed))


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_free_running_fp64_matches_oracle(oracle):
    """both sides run the same action sequence from reset; fp64 must track the oracle closely"""
    rng = np.random.default_rng(11)
    T = 60
    acts = rng.uniform(-1, 1, (T, 8 * A)).astype(np.float32)
    e = oracle.Env(A, K, 42, reward="progress", weights=(0.2, 0.4, 0.1, 0.4))
    e.reset()
    env = _gpu_env(1, "fp64")
    for t in range(T):
        ref_obs, ref_r, ref_term, _, info = e.step(acts[t])
        obs, rew, term, _ = env.step_tensors(torch.as_tensor(acts[t:t + 1], device=env.device))
        ctx = f"step {t}"
        assert bool(term.item()) == ref_term, ctx
        got = (env.terminal_obs if ref_term else obs)[0].cpu().numpy()
        np.testing.assert_allclose(got, ref_obs, rtol=1e-6, atol=1e-6, err_msg=ctx)
        np.testing.assert_allclose(rew.item(), ref_r, rtol=1e-5, atol=1e-5, err_msg=ctx)
        if ref_term:
            e.reset()
    env.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_full_size_properties():
    """4096 arenas (BASELINE config 2), fp32: finite, unit quaternions, deterministic, no capacity drops"""
    n = 4096
    env = _gpu_env(n, "fp32")
    g = torch.Generator(device=env.device)
    g.manual_seed(0)
    acts = [torch.rand(n, 8 * A, device=env.device, generator=g) * 2 - 1 for _ in range(12)]
    for a in acts:
        env.step_tensors(a)
    env.sync()
    s1 = env.get_state()
    obs1 = env.obs.clone()
    from factory_marl_amd import state as st

    nq, nv, nu, nd, ni = st.sizes(A, K)
    d = s1[:, :8 * nd].copy().view(np.float64)
    assert np.isfinite(d).all()
    q = d[:, :nq]
    for k in range(K):
        # unit quaternions, except a cube spawned by this env-step's TaskManager (pose (0, 1, 2) with the raw
        # U(0,1)^4 draw, task_utils.py:47-52) -- it is normalised on use and by its first integration
        qk = q[:, 1 + 7 * k:1 + 7 * k + 7]
        spawned = np.all(qk[:, :3] == [0.0, 1.0, 2.0], axis=1)
        qn = np.linalg.norm(qk[:, 3:], axis=1)
        assert np.all(np.abs(qn[~spawned] - 1) < 1e-4)
    assert env.counters()[:, 0].sum() == 0
    env.close()
    env2 = _gpu_env(n, "fp32")
    for a in acts:
        env2.step_tensors(a)
    env2.sync()
    assert torch.equal(obs1, env2.obs), "kernel is not deterministic"
    env2.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("A_,K_", [(2, 8), (2, 6)])  # compile-time FixedDims<2, 8>; runtime-dims kernel (K = 6)
def test_teacher_forced_fp64_other_configs(oracle, A_, K_):
    """same gate as the (2, 4) benchmark scene: fp64 within 1e-7 per env-step, integer state / flags exact"""
    traj = _rollout(oracle, A_, K_, 40, seed_actions=3)
    r = _compare(traj, "fp64", 1e-7, A_, K_)
    print(f"fp64 ({A_},{K_}): worst rel err {r['errs'].max():.3e}, obs {r['obs_err'].max():.2e}")
    assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
    assert r["errs"].max() <= 1e-7
    assert r["obs_err"].max() <= 1e-5 and r["rew_err"].max() <= 1e-6
    assert r["counters"][:, 0].sum() == 0


IK_CLASSES = ["FactoryManipulationEnv", "SingleFullRLProgressRewardEnv", "SingleDeltaProgressRewardEnv",
              "AllDeltaProgressRewardEnv", "PauseIKToggleEnv", "BackupIKToggleEnv"]


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("env_class", IK_CLASSES)
def test_teacher_forced_ik_classes_fp64(oracle, env_class):
    """the IK env classes (environments.py:25-248, 386-459, 498-645): the GPU IK base policy (FSM, targets,
    ignore maps, DLS IK) and class composition against the oracle -- IK state exact, proposals / state close"""
    traj = pu.rollout(oracle, A, K, 150, seed_actions=13, env_class=env_class)
    r = pu.compare(traj, "fp64", A, K, env_class, verbose_tol=1e-6)
    print(f"fp64 {env_class}: worst rel err {r['errs'].max():.3e}, obs {r['obs_err'].max():.2e}, "
          f"IK block {r['ik_err'].max():.2e}, terms {r['terms']}, post-reset worst "
          f"{r['reset_err'].max() if r['resets'] else 0:.2e}")
    assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
    assert r["resets"] == r["terms"] and not r["reset_bad"] and (r["resets"] == 0 or r["reset_err"].max() <= 1e-6)
    # grasps put the stiff gripper contacts (solref 0.002, gripper.xml) on a cube: the fp64 round-off of the
    # two implementations grows further there than in the AllFullRL episodes (measured worst 2.0e-6, Pause
    # toggle step 75, a cube's spin); the gate is 10x under the SURVEY's 1e-4
    assert r["errs"].max() <= 1e-5
    assert r["obs_err"].max() <= 1e-5 and r["rew_err"].max() <= 1e-6
    assert r["ik_err"].max() <= 1e-6


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("A_,K_,T,seed", [(2, 4, 300, 21), (2, 8, 300, 5), (2, 10, 250, 9)])
def test_teacher_forced_long_fp64(oracle, A_, K_, T, seed):
    """>= 250 env-steps from reset (every cube spawned, cube-cube contacts, force terminations with their
    auto-resets): fp64 within 1e-7 per env-step, integer state / RNG / scores / flags bit-exact"""
    traj = _rollout(oracle, A_, K_, T, seed_actions=seed)
    r = _compare(traj, "fp64", 1e-7, A_, K_)
    print(f"fp64 ({A_},{K_}) x {T}: worst {r['errs'].max():.3e}, terminations {r['terms']}, "
          f"max cubes {r['max_cubes']}, post-reset records {r['resets']} worst {r['reset_err'].max():.2e}")
    assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
    assert r["errs"].max() <= 1e-7
    # the record after a terminating env-step is the auto-reset one (TaskManager RNG continuing, task_utils.py:146-156,
    # environments.py:204-248): integers / RNG exact, float record and reset() observation close to the oracle's
    assert r["resets"] == r["terms"] >= 1 and not r["reset_bad"] and r["reset_err"].max() <= 1e-6
    assert r["obs_err"].max() <= 1e-5 and r["rew_err"].max() <= 1e-6
    assert r["counters"][:, 0].sum() == 0


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_fp32_other_scenes_within_survey_gate(oracle):
    """fp32 (2, 8) and (2, 10) compile-time scenes over long trajectories: integer state / flags exact, the
    SURVEY gate on >= 98.5 % / 99 % of env-steps (round 4: 99.0 % / 99.2 %) with the worst step capped (measured
    2.8e-3 / 3.07e-3 and 1.07e-3; against the 1e-8-tolerance oracle 100 % / 99.6 %, test below)"""
    for A_, K_, T, seed, gate, cap in [(2, 8, 300, 5, 0.985, 4e-3), (2, 10, 250, 9, 0.99, 1.5e-3)]:
        traj = _rollout(oracle, A_, K_, T, seed_actions=seed)
        r = _compare(traj, "fp32", 1e-4, A_, K_)
        frac = float(np.mean(r["errs"] <= 1e-4))
        print(f"fp32 ({A_},{K_}): {frac:.1%} of {len(r['errs'])} steps within 1e-4; median {np.median(r['errs']):.2e}, "
              f"worst {r['errs'].max():.2e}")
        assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
        assert frac >= gate and r["errs"].max() <= cap, (frac, r["errs"].max())
        assert frac >= _float_floor(A_, K_, T, seed)["within"]  # plain-float restatement: 53.5 % / 75.9 %


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_masked_reset_only_touches_masked_arenas():
    """fm_reset with a mask (env_method("reset", indices=...)): other arenas keep their state bit for bit"""
    env = _gpu_env(8, "fp32")
    g = torch.Generator(device=env.device)
    g.manual_seed(1)
    for _ in range(3):
        env.step_tensors(torch.rand(8, 8 * A, device=env.device, generator=g) * 2 - 1)
    env.sync()
    before = env.get_state()
    mask = np.zeros(8, np.uint8)
    mask[[1, 5]] = 1
    env.reset(mask=mask)
    env.sync()
    after = env.get_state()
    fresh = _gpu_env(1, "fp32").get_state()[0]
    for i in range(8):
        if mask[i]:
            from factory_marl_amd import state as st

            da, ia, _ = st.unpack(A, K, after[i])
            df, i_f, _ = st.unpack(A, K, fresh)
            nq = st.sizes(A, K)[0]
            assert np.array_equal(da[:nq], df[:nq])  # reset pose
        else:
            assert np.array_equal(after[i], before[i])
    env.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("env_class", ["BackupIKToggleEnv", "PauseIKToggleEnv"])
def test_config5_scene_4x16_fp32(oracle, env_class):
    """BASELINE config 5's arena (4 arms x 16 cubes, the toggle env classes, environments.py:580-645) in the
    benchmarked compile-time fp32 kernel, teacher-forced over 150 env-steps from reset against the float64 oracle and
    the oracle restepped at MuJoCo's 1e-8 Newton tolerance (one GPU launch): no contact dropped (the scene exceeds
    64), IK / task integer state exact, and per step the nearer of the two oracles within the SURVEY gate on >= 99 %
    of the steps and within 1e-3 on every step.  (Round 4: the Pause toggle's step 142 is a bifurcation where the
    1e-12 and the 1e-8 oracle differ by 0.92 relative; the kernel follows one of them, profiles/r04_parity.md)"""
    traj = pu.rollout(oracle, 4, 16, 150, seed_actions=3, env_class=env_class)
    tol8 = pu.restep_at_tolerance(oracle, 4, 16, traj, 1e-8, env_class)
    r = pu.compare(traj, "fp32", 4, 16, env_class, alt=tol8)
    e = r["errs"]
    print(f"fp32 (4,16) {env_class} vs the 1e-12 oracle: {np.mean(e <= 1e-4):.1%} within 1e-4, median "
          f"{np.median(e):.2e}, worst {e.max():.2e}, missing {list(r['err_steps'][e > 1e-4])}, max contacts "
          f"{int(r['counters'][:, 5].max())}, dropped {int(r['counters'][:, 0].sum())}")
    assert r["counters"][:, 0].sum() == 0 and r["counters"][:, 5].max() > 64
    assert not r["flag_bad"] and not r["int_bad"] and not r["reset_bad"], (r["flag_bad"], r["int_bad"])
    within, worst, missing = pu.two_oracle_gate(r, frac=0.99, cap=1e-3)
    print(f"  nearer of the two oracles: {within:.1%} within 1e-4, worst {worst:.2e}, missing {missing}")


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_config5_kernel_is_deterministic():
    """the (4,16) fp32 kernel (Hessian and contact records in global scratch, float atomics in the Hessian assembly)
    gives the same records when the same env-steps run twice"""
    out = []
    for _ in range(2):
        env = _gpu_env(256, "fp32", 4, 16, "PauseIKToggleEnv")
        g = torch.Generator(device=env.device)
        g.manual_seed(2)
        for _ in range(20):
            env.step_tensors((torch.rand(256, 4, device=env.device, generator=g) < 0.5).float())
        env.sync()
        out.append(env.get_state())
        env.close()
    assert np.array_equal(out[0], out[1])


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("env_class", ["PauseIKToggleEnv", "BackupIKToggleEnv"])
def test_teacher_forced_ik_classes_fp64_4x16(oracle, env_class):
    """BASELINE config 5's scene (4 arms x 16 cubes, environments.py:580-645, ik_policy.py:141-282) in the
    parity-grade fp64 build: since round 5 the compile-time FixedDims<4, 16> fp64 kernel (Hessian and contact records
    in the arena's global scratch block, the tree-block Newton solve in float64) -- the runtime DimsSpill kernel no
    longer runs it.  150 teacher-forced env-steps: IK FSM block and every integer exact, IK doubles within 1e-6, state
    within 1e-5"""
    traj = pu.rollout(oracle, 4, 16, 150, seed_actions=13, env_class=env_class)
    r = pu.compare(traj, "fp64", 4, 16, env_class, verbose_tol=1e-6)
    print(f"fp64 (4,16) {env_class}: worst rel err {r['errs'].max():.3e}, obs {r['obs_err'].max():.2e}, "
          f"IK block {r['ik_err'].max():.2e}, terms {r['terms']}, max contacts {int(r['counters'][:, 5].max())}")
    assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
    assert r["errs"].max() <= 1e-5
    assert r["obs_err"].max() <= 1e-5 and r["rew_err"].max() <= 1e-6
    assert r["ik_err"].max() <= 1e-6
    assert r["counters"][:, 0].sum() == 0


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("A_,K_,env_class", [(2, 4, "PauseIKToggleEnv"), (2, 4, "BackupIKToggleEnv"),
                                             (2, 4, "AllDeltaProgressRewardEnv"), (2, 8, "PauseIKToggleEnv"),
                                             (2, 10, "BackupIKToggleEnv"), (2, 10, "PauseIKToggleEnv")])
def test_fp32_ik_classes_within_survey_gate(oracle, A_, K_, env_class):
    """the IK classes (grasps: a cube held between the gripper plates' contacts) in the benchmarked fp32 kernels of
    the 2-arm scenes, 150 teacher-forced env-steps from reset against the float64 oracle and the oracle restepped at
    MuJoCo's 1e-8 tolerance: integer / IK state exact, the nearer oracle within the SURVEY gate on >= 99 % of the
    steps and within 5e-3 on every step (the cap of the fp32 (2,8) scene test above; measured round 6: (2,4) Backup
    step 111 at 4.2e-3 against both oracles, every other step within 1e-4).  Round 6: these kernels take float64 arm
    poses (FixedDims::f64ik) -- with the float arm chain the (2,4) Pause toggle had 87 % of its steps within, worst
    0.54 (host backend, same kernel)"""
    traj = pu.rollout(oracle, A_, K_, 150, seed_actions=3, env_class=env_class)
    tol8 = pu.restep_at_tolerance(oracle, A_, K_, traj, 1e-8, env_class)
    r = pu.compare(traj, "fp32", A_, K_, env_class, alt=tol8, verbose_tol=1e-3)
    e = r["errs"]
    print(f"fp32 ({A_},{K_}) {env_class} vs the 1e-12 oracle: {np.mean(e <= 1e-4):.1%} within 1e-4, median "
          f"{np.median(e):.2e}, worst {e.max():.2e}")
    assert not r["flag_bad"] and not r["int_bad"] and not r["reset_bad"], (r["flag_bad"], r["int_bad"])
    assert r["counters"][:, 0].sum() == 0
    within, worst, missing = pu.two_oracle_gate(r, frac=0.99, cap=5e-3)
    print(f"  nearer of the two oracles: {within:.1%} within 1e-4, worst {worst:.2e}, missing {missing}")


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_ik_timing_follows_control_frequency_and_pt_time(oracle):
    """ik_policy.py:56-67 derives the IK policy's step counts (release 0.5 s, grasp 1 s, move 1 s, timeout 3 s) and its
    velocity compensation (pt_time * dt * 15) from env.dt and env.pt_time: at control_frequency 20 Hz (frame_skip 50:
    10 / 20 / 20 / 60 env-steps) and pt_time 0.3 the GPU IK FSM stays exact with the oracle's"""
    kw = dict(pt_time=0.3, control_frequency=20)
    traj = pu.rollout(oracle, 2, 4, 300, seed_actions=13, env_class="PauseIKToggleEnv", env_kw=kw)
    r = pu.compare(traj, "fp64", 2, 4, "PauseIKToggleEnv", verbose_tol=1e-6, env_kwargs=kw)
    ints = np.stack([o["ints"] for o in traj[2]])
    states = set(ints[:, 2 * 4 + 11::5].ravel().tolist())
    print(f"20 Hz / pt_time 0.3: worst {r['errs'].max():.2e}, IK block {r['ik_err'].max():.2e}, states {sorted(states)}")
    assert {0, 1, 2, 3} <= states
    assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
    assert r["errs"].max() <= 1e-5 and r["ik_err"].max() <= 1e-6


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_wide_rerun_kernel_matches_oracle(trajectory, precision):
    """the (2,4) scene's wide-capacity rerun kernel (FixedDims<2, 4, true>, float64 for both builds) on every env-step
    of the 96-step trajectory (FM_FORCE_RERUN=1: the 64-contact launch abandons each arena at its first stage): the
    same gates as the 64-contact kernel -- fp64 within 1e-7, the fp32 handle (its abandoned env-steps stepped in
    float64 at MuJoCo's 1e-8 Newton tolerance) the SURVEY gate on >= 98.5 %, integer state exact"""
    r = pu.compare(trajectory, precision, A, K, experiment="FM_FORCE_RERUN=1")
    e = r["errs"]
    print(f"{precision} wide rerun: worst {e.max():.2e}, within 1e-4 {np.mean(e <= 1e-4):.1%}, reruns "
          f"{int(r['counters'][:, 8].sum())}")
    assert not r["flag_bad"] and not r["int_bad"], (r["flag_bad"], r["int_bad"])
    assert int(r["counters"][:, 8].sum()) == len(trajectory[0])  # every arena went through the wide kernel
    if precision == "fp64":
        assert e.max() <= 1e-7 and r["obs_err"].max() <= 1e-5 and r["rew_err"].max() <= 1e-6
    else:
        assert np.mean(e <= 1e-4) >= 0.985 and e.max() <= 5e-4


def _crowded_states(oracle, n_states, lo=66, hi=110, seed=0):
    """(2,4) records whose first stage holds lo..hi contacts: the cubes landed at their parking spots (16 floor
    contacts), then both arms set (qpos and the stage positions, at rest) to random joint poses that reach into the
    table, the belt and each other -- counted by the oracle's own collision at that pose"""
    from factory_marl_amd import state as st

    e = oracle.Env(A, K, 42, weights=(0.2, 0.4, 0.1, 0.4))
    e.reset()
    for _ in range(8):
        e.step(np.zeros(8 * A, np.float32))
    d0, i0, r0 = e.export_state()
    nq, nv = st.sizes(A, K)[:2]
    a0 = 1 + 7 * K
    rng = np.random.default_rng(seed)
    recs = []
    for _ in range(4000):
        q = d0[:nq].copy()
        for arm in range(A):
            b = a0 + 9 * arm
            q[b:b + 7] = [rng.uniform(-1, 1), rng.uniform(-2.09, 2.09), rng.uniform(-1, 1), rng.uniform(-2.09, 2.09),
                          rng.uniform(-1, 1), rng.uniform(-2.09, 2.09), 0.0]
        e.data.qpos[:] = q
        e.data.forward()
        if lo <= e.data.ncon <= hi:
            d = d0.copy()
            d[:nq] = q  # qpos
            d[nq + nv:2 * nq + nv] = q  # the stage the env-step's first mj_step1 sees
            d[nq:nq + nv] = 0.0
            d[2 * nq + nv:2 * nq + 2 * nv] = 0.0
            recs.append(st.pack(A, K, d, i0, r0))
            if len(recs) == n_states:
                break
    return np.stack(recs)


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_wide_rerun_resumes_at_the_abandoned_substep(trajectory, precision):
    """an env-step abandoned by the 64-contact kernel after substep 0 is resumed by the wide kernel at that substep
    from the saved substep state (State::resume: master state, warmstart, low-pass control, clipped control target,
    the stages' contact counters) instead of being redone.  FM_RERUN_AT_50=1 abandons every env-step of the 96-step
    trajectory at substep 50: the result must meet the same gates as the uninterrupted kernel (fp64 within 1e-7,
    fp32 the SURVEY gate on >= 98.5 %, integer state and flags exact)"""
    r = pu.compare(trajectory, precision, A, K, experiment="FM_RERUN_AT_50=1")
    e = r["errs"]
    # the episode-mix counters of the resumed env-steps: contacts summed over the stages (ctr[4]: stage 50 is counted
    # once, by the wide kernel that redoes it) and the largest stage (ctr[5]), against the uninterrupted kernel
    ref = pu.compare(trajectory, precision, A, K)
    same4 = float(np.mean(r["counters"][:, 4] == ref["counters"][:, 4]))
    print(f"{precision} resumed at substep 50: worst {e.max():.2e}, within 1e-4 {np.mean(e <= 1e-4):.1%}, reruns "
          f"{int(r['counters'][:, 8].sum())}, contact sums equal to the uninterrupted run's on {same4:.1%} of arenas")
    assert not r["flag_bad"] and not r["int_bad"] and not r["reset_bad"], (r["flag_bad"], r["int_bad"], r["reset_bad"])
    assert int(r["counters"][:, 8].sum()) == len(trajectory[0])
    if precision == "fp64":
        assert np.array_equal(r["counters"][:, 4], ref["counters"][:, 4])
        assert np.array_equal(r["counters"][:, 5], ref["counters"][:, 5])
    else:  # the fp32 handle's stages 50-99 run in float64 here: a marginal contact may differ, not a whole stage's
        assert same4 >= 0.9 and np.abs(r["counters"][:, 4] - ref["counters"][:, 4]).max() <= 8
    if precision == "fp64":
        assert e.max() <= 1e-7 and r["obs_err"].max() <= 1e-5 and r["rew_err"].max() <= 1e-6
    else:
        assert np.mean(e <= 1e-4) >= 0.985 and e.max() <= 5e-4


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_wide_rerun_resume_ik_class_fp64(oracle):
    """the resume path of an IK class (PauseIKToggleEnv): the compose and the toggles' pause_last writes happened in
    the 64-contact launch and stand (no record backup restored), the wide kernel continues at substep 50"""
    traj = pu.rollout(oracle, A, K, 120, seed_actions=13, env_class="PauseIKToggleEnv")
    r = pu.compare(traj, "fp64", A, K, "PauseIKToggleEnv", experiment="FM_RERUN_AT_50=1")
    e = r["errs"]
    print(f"fp64 PauseIKToggleEnv resumed at substep 50: worst {e.max():.2e}, IK block {r['ik_err'].max():.2e}")
    assert not r["flag_bad"] and not r["int_bad"] and not r["reset_bad"], (r["flag_bad"], r["int_bad"], r["reset_bad"])
    assert int(r["counters"][:, 8].sum()) == len(traj[0])
    assert e.max() <= 1e-5 and r["ik_err"].max() <= 1e-6


def _calm_crowded_states(oracle, n_states, seed=1):
    """(2,4) records whose first stage holds 66-100 contacts without a force termination: the arms moved from the
    parked pose towards a random pose that reaches into the table / belt / each other only as far as the contact
    count needs (bisection on the path to a target count), at rest, with the control target and the actions holding
    that pose -- so the env-step is compared as a state, not only through its terminal observation.  Kept when the
    oracle's env-step from it does not terminate.  Returns (records, actions)"""
    from factory_marl_amd import state as st

    e = oracle.Env(A, K, 42, weights=(0.2, 0.4, 0.1, 0.4))
    e.reset()
    for _ in range(8):
        e.step(np.zeros(8 * A, np.float32))
    d0, i0, r0 = e.export_state()
    nq, nv = st.sizes(A, K)[:2]
    a0 = 1 + 7 * K
    lim = np.asarray(e.model.ctrlrange).reshape(-1, 2)
    off = 2 * nq + 3 * nv  # ctrl_target in the float64 record
    base = d0[:nq].copy()
    rng = np.random.default_rng(seed)

    def ncon(q):
        e.data.qpos[:] = q
        e.data.forward()
        return e.data.ncon

    recs, acts = [], []
    for _ in range(20000):
        q = base.copy()
        for arm in range(A):
            b = a0 + 9 * arm
            q[b:b + 7] = [rng.uniform(-1, 1), rng.uniform(-2.09, 2.09), rng.uniform(-1, 1), rng.uniform(-2.09, 2.09),
                          rng.uniform(-1, 1), rng.uniform(-2.09, 2.09), 0.0]
        target = int(rng.integers(66, 90))
        if ncon(q) < target:
            continue
        lo_t, hi_t = 0.0, 1.0
        for _ in range(12):
            m = 0.5 * (lo_t + hi_t)
            lo_t, hi_t = (lo_t, m) if ncon(base + m * (q - base)) >= target else (m, hi_t)
        qc = base + hi_t * (q - base)
        if not 66 <= ncon(qc) <= 100:
            continue
        d = d0.copy()
        d[:nq] = qc
        d[nq + nv:2 * nq + nv] = qc
        d[nq:nq + nv] = 0.0
        d[2 * nq + nv:2 * nq + 2 * nv] = 0.0
        a = np.zeros(8 * A, np.float32)
        for arm in range(A):
            for j in range(8):
                lo_, hi_ = lim[1 + 8 * arm + j]
                qq = qc[a0 + 9 * arm + j] if j < 7 else d[off + 1 + 8 * arm + j]
                d[off + 1 + 8 * arm + j] = qq
                a[8 * arm + j] = np.arctanh(np.clip(2 * (qq - lo_) / (hi_ - lo_) - 1, -0.999999, 0.999999))
        rec = st.pack(A, K, d, i0, r0)
        e.import_state(*st.unpack(A, K, rec))
        if e.step(a)[2]:
            continue  # force termination: not a calm state
        recs.append(rec)
        acts.append(a)
        if len(recs) == n_states:
            break
    return np.stack(recs), np.stack(acts)


def _crowded_trajectory(oracle):
    """12 crowded records (arms deep in the table: most force-terminate) + 10 calm ones (compared as states)"""
    recs = _crowded_states(oracle, 12)
    acts = np.random.default_rng(4).uniform(-1, 1, (len(recs), 8 * A)).astype(np.float32)
    crec, cact = _calm_crowded_states(oracle, 10)
    recs, acts = np.concatenate([recs, crec]), np.concatenate([acts, cact])
    return pu.restep_at_tolerance(oracle, A, K, (recs, acts, None), 0.0)


@pytest.fixture(scope="module")
def crowded(oracle):
    traj = _crowded_trajectory(oracle)
    return traj, pu.restep_at_tolerance(oracle, A, K, traj, 1e-8)


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_contacts_above_64_are_not_dropped(crowded, precision):
    """(2,4) benchmark scene, env-steps whose stages hold more than 64 contacts (arms reaching into the table, the belt
    and each other; the parked cubes' 16 floor contacts): the 64-contact launch abandons them and the (float64) wide
    kernel steps them -- no contact is dropped, and from the same records the oracle (which keeps every contact,
    base_env.py:217-218 -> mj_step) gives the same result.  >= 8 of the records do not terminate, so they are
    compared as states: fp64 within 1e-7; the fp32 handle (the benchmarked build, whose abandoned env-steps run in
    float64 at MuJoCo's 1e-8 Newton tolerance) at the SURVEY gate against the nearer of the 1e-12 / 1e-8 oracles on
    >= 99 % of the states and within 1e-3 on every one; integer state / flags exact in both"""
    traj, tol8 = crowded
    recs = traj[0]
    r = pu.compare(traj, precision, A, K, alt=tol8 if precision == "fp32" else None, verbose_tol=1e-4)
    e = r["errs"]
    print(f"{precision} >64-contact env-steps: {len(recs)}, compared {len(e)} (+{r['terms']} terminations), worst "
          f"{e.max() if len(e) else 0:.2e}, reruns {int(r['counters'][:, 8].sum())}, max contacts "
          f"{int(r['counters'][:, 5].max())}, dropped {int(r['counters'][:, 0].sum())}")
    assert len(recs) == 22 and int(r["counters"][:, 5].max()) > 64 and int(r["counters"][:, 0].sum()) == 0
    assert int(r["counters"][:, 8].sum()) == len(recs)  # each one went through the wide kernel
    assert not r["flag_bad"] and not r["int_bad"] and not r["reset_bad"], (r["flag_bad"], r["int_bad"], r["reset_bad"])
    assert len(e) >= 8  # compared as states, not only through their terminal observations
    if precision == "fp64":
        assert e.max() <= 1e-7
        assert r["obs_err"].max() <= 1e-5
    else:
        # round 5 stepped these in float32 (a float32 Hessian of 60-100 stiff contacts with the gripper plates' small
        # masses among them: 8 of 12 states within the gate, worst 2.7e-2); the abandoned env-steps now run in float64
        within, worst, missing = pu.two_oracle_gate(r, frac=0.99, cap=1e-3)
        print(f"  nearer of the two oracles: {within:.1%} within 1e-4, worst {worst:.2e}, missing {missing}")


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("env_class", ["PauseIKToggleEnv", "AllDeltaProgressRewardEnv"])
def test_wide_rerun_kernel_ik_classes_fp64(oracle, env_class):
    """the rerun path of the IK classes (FM_FORCE_RERUN=1: every (2,4) env-step abandoned by the 64-contact kernel
    after its IK compose wrote the FSM / toggle blocks, then restored from State::bak and stepped by the wide kernel)
    against the oracle in fp64 with the gates of the 64-contact kernel's IK-class test: IK FSM block and every integer
    exact, IK doubles within 1e-6, state within 1e-5 (grasps put the stiff gripper contacts on a cube)"""
    traj = pu.rollout(oracle, A, K, 120, seed_actions=13, env_class=env_class)
    r = pu.compare(traj, "fp64", A, K, env_class, experiment="FM_FORCE_RERUN=1")
    e = r["errs"]
    print(f"fp64 wide rerun {env_class}: worst {e.max():.2e}, IK block {r['ik_err'].max():.2e}, reruns "
          f"{int(r['counters'][:, 8].sum())}, terms {r['terms']}")
    assert not r["flag_bad"] and not r["int_bad"] and not r["reset_bad"], (r["flag_bad"], r["int_bad"], r["reset_bad"])
    assert int(r["counters"][:, 8].sum()) == len(traj[0])
    assert e.max() <= 1e-5 and r["ik_err"].max() <= 1e-6
    assert r["obs_err"].max() <= 1e-5 and r["rew_err"].max() <= 1e-6
