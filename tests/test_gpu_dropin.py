"""The SB3 drop-in surface on the GPU path and BASELINE config 3 at full size.

* src/learning.py:98-100's make_vec_env line with vec_env_cls=FactoryVecEnv (CONFIG of learning.py:20-48);
* VecEnv.set_attr / get_attr on the reference env's runtime attributes (base_env.py:133-147) and env_method;
* config 3: 16384 arenas of the 2 x 8 scene stepped at full size (properties), and one PPO iteration on that
  scene (rollout + update)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import pathlib  # noqa: E402

_FIX = pathlib.Path(__file__).resolve().parent / "golden" / "runs_fixtures.npz"


def _have_gpu():
    return torch.cuda.is_available()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_learning_py_make_vec_env_line_on_gpu():
    from factory_marl_amd import FactoryVecEnv, Monitor, environments, make_vec_env

    CONFIG = dict(num_envs=8, env_class="PauseIKToggleEnv",
                  env_kwargs={"num_arms": 4, "render_mode": "rgb_array", "seed": 42, "initial_conveyor_speed": 0.1,
                              "conveyor_acceleration": 0.001, "pt_time": 0.2, "force_contact_threshold": 200.0,
                              "max_num_objects": 10, "control_frequency": 10, "spawn_freq": 1 / 10,
                              "spawn_freq_increase": 1.001})
    env = make_vec_env(lambda: Monitor(getattr(environments, CONFIG["env_class"])(**CONFIG["env_kwargs"])),
                       n_envs=CONFIG["num_envs"], vec_env_cls=FactoryVecEnv)
    obs = env.reset()
    assert isinstance(obs, np.ndarray) and obs.shape == (8, 24 * 4 + 13 * 10 + 8 * 4)
    # the toggle classes' rows are float64 as in the reference (environments.py:576; the saved run y6lp1j7k's
    # SB3 _last_obs is float64 [8, 258], tests/golden/runs_fixtures.npz)
    fx = np.load(_FIX, allow_pickle=False)
    ref = fx["last_obs_y6lp1j7k"]
    assert obs.dtype == np.float64 and ref.dtype == obs.dtype and ref.shape == obs.shape
    assert env.action_space.nvec.tolist() == [2] * 4
    rng = np.random.default_rng(0)
    for _ in range(5):
        obs, rew, done, infos = env.step(rng.integers(0, 2, (8, 4)))
    assert isinstance(rew, np.ndarray) and rew.shape == (8,) and done.dtype == bool and len(infos) == 8
    assert all("scores" in i for i in infos)
    assert env.get_attr("ep_score_history") == [[] for _ in range(8)] or len(env.get_attr("ep_score_history")) == 8
    env.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("env_class", ["PauseIKToggleEnv", "BackupIKToggleEnv"])
def test_toggle_observation_rows_are_float64(env_class):
    """IKTogglingEnv._process_observation (environments.py:560-577) concatenates the float32 state columns with the
    float64 IK proposals: the GPU env's rows are float64, the state columns are the float32 values widened exactly,
    the proposal columns carry the arena record's float64 ik_actions bit for bit; obs_dtype="float32" gives the
    rounded rows"""
    from factory_marl_amd import FactoryVecEnv, state as st
    from factory_marl_amd.environments import run_kwargs

    n, A, K = 16, 2, 4
    kw = run_kwargs(env_class, num_arms=A, max_num_objects=K, seed=42)
    e64 = FactoryVecEnv(n, env_class=env_class, env_kwargs=kw, return_numpy=False)
    e32 = FactoryVecEnv(n, env_class=env_class, env_kwargs=kw, return_numpy=False, obs_dtype="float32")
    for e in (e64, e32):
        e.reset()
    g = torch.Generator(device=e64.device)
    g.manual_seed(5)
    for _ in range(30):
        a = (torch.rand(n, A, device=e64.device, generator=g) < 0.5).float()
        o64 = e64.step_tensors(a)[0].clone()
        o32 = e32.step_tensors(a)[0].clone()
    assert o64.dtype == torch.float64 and o32.dtype == torch.float32
    o64, o32 = o64.cpu().numpy(), o32.cpu().numpy()
    ns = 24 * A + 13 * K
    assert np.array_equal(o64[:, :ns], o32[:, :ns].astype(np.float64))  # widened float32 columns
    assert np.array_equal(o64[:, ns:].astype(np.float32), o32[:, ns:])
    recs = e64.get_state()
    for i in range(n):
        d, _, _ = st.unpack(A, K, recs[i])
        ik = np.array([d[len(d) - 27 * A + 27 * a + 11 + j] for a in range(A) for j in range(8)])
        assert np.array_equal(o64[i, ns:], ik)  # the float64 proposals, unrounded
    assert np.abs(o64[:, ns:] - o64[:, ns:].astype(np.float32)).max() > 0  # they do carry bits beyond float32
    e64.close()
    e32.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_set_attr_get_attr_env_method():
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    n = 4
    env = FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42))
    env.reset()
    assert env.get_attr("conveyor_acceleration") == [0.001] * n
    assert env.get_attr("base_reward") == [0.4] * n
    env.set_attr("conveyor_acceleration", 0.5)
    env.set_attr("play_time", 5.0, indices=[1])
    env.set_attr("conveyor_speed", 0.2, indices=[2])
    assert env.get_attr("play_time") == [0.0, 5.0, 0.0, 0.0]
    zero = np.zeros((n, 16), np.float32)
    env.step(zero)
    pt = env.play_time.cpu().numpy()
    cs = env.conveyor_speed.cpu().numpy()
    np.testing.assert_allclose(pt, [0.1, 5.1, 0.1, 0.1], rtol=0, atol=1e-12)
    # base_env.py:269: speed += acceleration * dt with the new acceleration
    np.testing.assert_allclose(cs, [0.1 + 0.05, 0.1 + 0.05, 0.2 + 0.05, 0.1 + 0.05], rtol=0, atol=1e-12)
    with pytest.raises(ValueError):
        env.set_attr("num_arms", 4)
    with pytest.raises(ValueError):
        env.set_attr("conveyor_acceleration", 0.3, indices=[0])  # one value per batch
    env.set_attr("tag", "x", indices=[0])
    assert env.get_attr("tag", indices=[0]) == ["x"]
    out = env.env_method("reset", indices=[2])
    assert len(out) == 1 and out[0][0].shape == (env.obs_dim,) and out[0][1] == {}
    img = env.env_method("render", indices=[0, 3], width=64, height=48)
    assert len(img) == 2 and img[0].shape == (48, 64, 3)
    with pytest.raises(AttributeError):
        env.env_method("step_sim")
    env.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_config3_scene_full_size_properties():
    """BASELINE config 3 at full size: 16384 arenas of the 2 x 8 scene, random actions: finite state, unit
    quaternions, no contact dropped for capacity, deterministic"""
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd import state as st
    from factory_marl_amd.environments import run_kwargs

    A, K, n = 2, 8, 16384
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    acts = [torch.rand(n, 8 * A, device="cuda", generator=g) * 2 - 1 for _ in range(10)]
    outs = []
    for _ in range(2):
        env = FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=A, max_num_objects=K,
                                                       seed=42), return_numpy=False)
        env.reset()
        for a in acts:
            env.step_tensors(a)
        env.sync()
        s = env.get_state()
        assert env.counters()[:, 0].sum() == 0
        outs.append(env.obs.clone())
        env.close()
    nq, nv, nu, nd, ni = st.sizes(A, K)
    d = s[:, :8 * nd].copy().view(np.float64)
    assert np.isfinite(d).all()
    q = d[:, :nq]
    for k in range(K):
        qk = q[:, 1 + 7 * k:1 + 7 * k + 7]
        spawned = np.all(qk[:, :3] == [0.0, 1.0, 2.0], axis=1)
        assert np.all(np.abs(np.linalg.norm(qk[:, 3:], axis=1)[~spawned] - 1) < 1e-4)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_ppo_iteration_on_config3_scene():
    """one PPO iteration (rollout of 8 env-steps + 4 epochs of updates) on 2048 arenas of the 2 x 8 scene"""
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs
    from factory_marl_amd.ppo import PPO

    env = FactoryVecEnv(2048, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=8,
                                                      seed=42), return_numpy=False)
    ppo = PPO(env, n_steps=8, batch_size=4096, n_epochs=4, seed=0)
    ppo.learn(2048 * 8)
    rec = ppo.logs[-1]
    assert rec["timesteps"] == 2048 * 8
    for k in ("policy_loss", "value_loss", "entropy_loss"):
        assert np.isfinite(rec[k])
    assert np.isfinite(rec["reward_per_step"])
    env.close()
