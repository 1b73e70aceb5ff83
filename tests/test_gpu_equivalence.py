"""The kernel's exact reformulations against their straightforward forms, on the GPU (experiment switches set on a
live handle of the experiment build, FactoryVecEnv(..., experimental=True).set_experiment; the product library is
compiled without them, and test_product_equals_experiment_build holds the two builds to the same bits):

* the cached midphase (a body-pair list of an inflated test reused across substeps) against a rebuild at every
  substep (FM_NO_MIDCACHE=1): the contact set is the same by construction, so the trajectories are bit-identical;
* the wave-parallel box-box narrowphase (SAT axes and clipping candidates over 16 lanes per pair) against one lane per
  pair (FM_SERIAL_BOXBOX=1): the same arithmetic per axis / candidate, bit-identical in fp32 (fp64: to rounding);
* the (4,16) scene's tree-block Newton solve (single trees factored per lane, the coupled trees + belt as one small
  dense system) against the dense blocked matrix-core Cholesky of the whole Hessian (FM_NO_TREEBLK=1) and against the
  sparse LDS one (FM_CHOL_LDS=2): the same factorisation up to float32 rounding order, so one env-step from the same
  state agrees to the SURVEY gate."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _have_gpu():
    return torch.cuda.is_available()


def _run(A, K, n, steps, switch, precision="fp32", env_class="AllFullRLProgressRewardEnv", value="1"):
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    env = FactoryVecEnv(n, env_class=env_class, env_kwargs=run_kwargs(env_class, num_arms=A, max_num_objects=K,
                                                                      seed=42),
                        precision=precision, seeds=42 + np.arange(n), return_numpy=False, experimental=True)
    env.reset()
    s0 = env.get_state()  # both runs start from this record (reset() continues the TaskManager RNG)
    g = torch.Generator(device=env.device)
    g.manual_seed(5)
    acts = [torch.rand(n, env.act_dim, device=env.device, generator=g) * 2 - 1 for _ in range(steps)]
    out = []
    for on in (False, True):
        env.set_state(s0)
        env.set_experiment(f"{switch}={value}" if on else "")
        for a in acts:
            env.step_tensors(a)
        env.sync()
        out.append(env.get_state())
    env.close()
    return out


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("A,K", [(2, 4), (2, 8)])
def test_cached_midphase_is_exact(A, K):
    a, b = _run(A, K, 256, 40, "FM_NO_MIDCACHE")
    assert np.array_equal(a, b)


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_parallel_box_box_is_exact():
    a, b = _run(2, 4, 256, 40, "FM_SERIAL_BOXBOX", precision="fp32")
    assert np.array_equal(a, b)


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_parallel_box_box_fp64_to_rounding():
    """fp64: the two code paths are inlined into different contexts and the compiler contracts a few multiply-adds
    differently, so they agree to float64 rounding rather than bit for bit (40 env-steps of 256 arenas: measured
    3.2e-11 relative, tools/boxbox_probe.py)"""
    import parity_util as pu
    from factory_marl_amd import state as st

    a, b = _run(2, 4, 256, 40, "FM_SERIAL_BOXBOX", precision="fp64")
    worst = max(max(m.max() for m in pu.state_err(2, 4, st.unpack(2, 4, a[i])[0], st.unpack(2, 4, b[i])[0]))
                for i in range(len(a)))
    print(f"parallel vs serial box-box, fp64, 40 env-steps: worst relative state difference {worst:.2e}")
    assert worst <= 1e-9


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("other", ["FM_NO_TREEBLK=1", "FM_CHOL_LDS=2"])
def test_treeblock_solve_agrees_with_dense_and_sparse_4x16(other):
    import parity_util as pu
    from factory_marl_amd import state as st

    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    A, K, n = 4, 16, 128
    env = FactoryVecEnv(n, env_class="PauseIKToggleEnv", env_kwargs=run_kwargs("PauseIKToggleEnv", num_arms=A,
                                                                               max_num_objects=K, seed=42),
                        seeds=42 + np.arange(n), return_numpy=False, experimental=True)
    env.reset()
    g = torch.Generator(device=env.device)
    g.manual_seed(9)
    for _ in range(40):  # contacts, grasps, cubes on the belt
        env.step_tensors((torch.rand(n, A, device=env.device, generator=g) < 0.5).float())
    env.sync()
    s0 = env.get_state()
    a = (torch.rand(n, A, device=env.device, generator=g) < 0.5).float()
    res = []
    for mode in ("", other):
        env.set_experiment(mode)
        env.set_state(s0)
        env.step_tensors(a)
        env.sync()
        res.append(env.get_state())
    env.close()
    errs = []
    for i in range(n):
        da = st.unpack(A, K, res[0][i])[0]
        db = st.unpack(A, K, res[1][i])[0]
        qd, vd = pu.state_err(A, K, da, db)
        errs.append(max(qd.max(), vd.max()))
    errs = np.array(errs)
    print(f"tree-block solve vs {other}, one env-step from 128 states: median {np.median(errs):.2e}, "
          f"within 1e-4 {np.mean(errs <= 1e-4):.1%}, worst {errs.max():.2e}")
    assert np.mean(errs <= 1e-4) >= 0.9 and np.median(errs) <= 1e-5


def _one_step(A, K, n, pre, switch, value="1", precision="fp32", base=""):
    """`pre` random-action env-steps from reset (n arenas of their own seeds: diverse states), then one env-step from
    that record with the switch off and on (on top of the `base` switches); returns the per-arena worst relative state
    difference (SURVEY metric)"""
    import parity_util as pu
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd import state as st
    from factory_marl_amd.environments import run_kwargs

    env = FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=A, max_num_objects=K, seed=42),
                        precision=precision, seeds=42 + np.arange(n), return_numpy=False, experimental=True)
    env.reset()
    g = torch.Generator(device=env.device)
    g.manual_seed(11)
    for _ in range(pre):
        env.step_tensors(torch.rand(n, env.act_dim, device=env.device, generator=g) * 2 - 1)
    env.sync()
    s0 = env.get_state()
    a = torch.rand(n, env.act_dim, device=env.device, generator=g) * 2 - 1
    res = []
    for on in (False, True):
        env.set_experiment(f"{base} {switch}={value}" if on else base)
        env.set_state(s0)
        env.step_tensors(a)
        env.sync()
        res.append(env.get_state())
    env.close()
    errs = np.array([max(m.max() for m in pu.state_err(A, K, st.unpack(A, K, res[0][i])[0],
                                                       st.unpack(A, K, res[1][i])[0])) for i in range(n)])
    return errs


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("A,K", [(2, 8), (2, 10)])
def test_two_pass_arrowhead_agrees_with_bordered_factor(A, K):
    """fp32 (2,8) / (2,10), dense-Hessian path (FM_NO_TREEBLK=1): the two-pass arrowhead block factor (chol_arrow2_rl,
    that path's default on arrowhead substeps) against the bordered register + matrix-core Schur factor
    (FM_NO_ARROW=1) -- the same Cholesky of the same Hessian in another summation order: one env-step from 256 diverse
    states agrees to float32 rounding"""
    errs = _one_step(A, K, 256, 60, "FM_NO_ARROW", base="FM_NO_TREEBLK=1")
    print(f"({A},{K}) two-pass arrowhead vs bordered factor, one env-step from 256 states: median {np.median(errs):.2e}, "
          f"99th pct {np.quantile(errs, 0.99):.2e}, worst {errs.max():.2e}")
    assert np.median(errs) <= 1e-6 and np.mean(errs <= 1e-5) >= 0.99 and errs.max() <= 1e-4


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("A,K", [(2, 8), (2, 10)])
def test_treeblock_solve_agrees_with_dense_path(A, K):
    """fp32 (2,8) / (2,10): the tree-block Newton solve (the default) against the dense global-block Hessian with its
    arrowhead / bordered factors (FM_NO_TREEBLK=1) -- the same system in another summation order"""
    errs = _one_step(A, K, 256, 60, "FM_NO_TREEBLK")
    print(f"({A},{K}) tree-block vs dense path, one env-step from 256 states: median {np.median(errs):.2e}, "
          f"99th pct {np.quantile(errs, 0.99):.2e}, worst {errs.max():.2e}")
    assert np.median(errs) <= 1e-6 and np.mean(errs <= 1e-5) >= 0.99 and errs.max() <= 1e-4


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("precision,A,K", [("fp32", 2, 4), ("fp64", 2, 4), ("fp32", 2, 8)])
def test_product_equals_experiment_build(precision, A, K):
    """the product library (no switches: FM_EXPERIMENTS=0, every switch branch compiled out) and the experiment build
    with every switch off step the same records to the same bits: the equivalence tests above, run on the experiment
    build, speak for the product kernels"""
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    n, steps = 256, 30
    out = []
    for exp in (False, True):
        env = FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=A, max_num_objects=K,
                                                     seed=42),
                            precision=precision, seeds=42 + np.arange(n), return_numpy=False, experimental=exp)
        env.reset()
        g = torch.Generator(device=env.device)
        g.manual_seed(3)
        for _ in range(steps):
            env.step_tensors(torch.rand(n, env.act_dim, device=env.device, generator=g) * 2 - 1)
        env.sync()
        out.append((env.get_state(), env.counters()))
        env.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
