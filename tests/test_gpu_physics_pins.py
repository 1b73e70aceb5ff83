"""The HIP env-step against MuJoCo's own outputs held by the reference (tests/test_physics_pins.py for the oracle):
free fall after a spawn, the resting depth of cubes on the belt and on the table, and the belt-carried velocity,
to float32 resolution -- through the C ABI, in both builds (fp32: float physics over the float64 master state)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_physics_pins as pins  # noqa: E402

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

A, K = pins.A, pins.K


def _have_gpu():
    return torch.cuda.is_available()


ref = pins.ref


def _gpu_still_run(precision, steps=299):
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd import state as st
    from factory_marl_amd.environments import run_kwargs

    env = FactoryVecEnv(1, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=A, max_num_objects=K, seed=42),
                        precision=precision)
    env.reset()
    nq, nv = 1 + 7 * K + 9 * A, 1 + 6 * K + 9 * A
    zero = torch.zeros(1, 8 * A, device=env.device)
    out = []
    for t in range(1, steps + 1):
        env.step_tensors(zero)
        d, _, _ = st.unpack(A, K, env.get_state()[0])
        out.append(dict(t=t, q=d[:nq].copy(), v=d[nq:nq + nv].copy()))
    env.close()
    return out


@pytest.fixture(scope="module", params=["fp64", "fp32"])
def gpu_run(request):
    if not _have_gpu():
        pytest.skip("needs an MI355X")
    return request.param, _gpu_still_run(request.param)


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_gpu_free_fall_after_spawn(ref, gpu_run):
    pins.check_free_fall(ref, gpu_run[1])


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_gpu_resting_depth_on_the_belt(ref, gpu_run):
    pins.check_belt_depth(ref, gpu_run[1])


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_gpu_belt_carried_velocity(ref, gpu_run):
    pins.check_carried_velocity(ref, gpu_run[1])


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_gpu_resting_depth_on_the_table(ref, precision):
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd import state as st
    from factory_marl_amd.environments import run_kwargs

    sizes = ref["sizes"]
    env = FactoryVecEnv(1, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=A, max_num_objects=K, seed=42),
                        precision=precision)
    env.reset()
    d, i, r = st.unpack(A, K, env.get_state()[0])
    env.set_state(st.pack(A, K, pins.table_start(d, sizes), i, r)[None])
    zero = torch.zeros(1, 8 * A, device=env.device)
    for _ in range(30):
        env.step_tensors(zero)
    z = st.unpack(A, K, env.get_state()[0])[0][1 + 7 * pins.TABLE_CUBE + 2]
    env.close()
    depth = 1.0 + sizes[pins.TABLE_CUBE] - z
    for ref_depth in pins.table_rows(ref):
        assert abs(depth - ref_depth) <= 1.0 * pins.ULP_Z, (precision, depth, ref_depth)
