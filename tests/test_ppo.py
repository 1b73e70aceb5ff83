"""PPO trainer (factory_marl_amd/ppo.py) on CPU: SB3-compatible policy layout against the reference's own
checkpoints, GAE against a plain restatement of SB3's RolloutBuffer, learning on a toy env, and the
data-parallel collectives under gloo with world size 2."""
import json
import os
import socket

import numpy as np
import pytest
import torch

from factory_marl_amd.ppo import PPO, ActorCriticPolicy, compute_gae, flat_allreduce, gae_reference

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class _Box:
    def __init__(self, n):
        self.shape = (n,)


class _MD:
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec)
        self.shape = self.nvec.shape


class ToyEnv:
    """FactoryVecEnv surface on CPU tensors: reward = -|a - target|^2, episodes of 8 steps"""

    def __init__(self, n=64, act_dim=3, discrete=False, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.num_envs, self.obs_dim, self.act_dim = n, 5, act_dim
        self.device = torch.device("cpu")
        self.action_space = _MD([2] * act_dim) if discrete else _Box(act_dim)
        self.discrete = discrete
        self.obs = torch.randn(n, 5, generator=g)
        self.t = torch.zeros(n)
        self.ep_return = torch.zeros(n, dtype=torch.float64)
        self._ret = torch.zeros(n, dtype=torch.float64)
        self.target = torch.full((act_dim,), 0.5) if not discrete else torch.ones(act_dim)
        self.g = g

    def reset(self):
        return self.obs

    def step_tensors(self, a):
        r = -((a - self.target) ** 2).sum(1)
        self._ret += r.double()
        self.t += 1
        done = self.t >= 8
        self.ep_return = torch.where(done, self._ret, self.ep_return)
        self._ret = torch.where(done, torch.zeros_like(self._ret), self._ret)
        self.t = torch.where(done, torch.zeros_like(self.t), self.t)
        self.obs = torch.randn(self.num_envs, 5, generator=self.g)
        z = torch.zeros(self.num_envs, dtype=torch.uint8)
        return self.obs, r, done.to(torch.uint8), z


@pytest.mark.parametrize("run", ["rk5rxnav", "y6lp1j7k"])
def test_policy_layout_matches_reference_checkpoints(run):
    """the reference's trained policies (runs/*.zip policy.pth, kept as data fixtures) load into
    ActorCriticPolicy unchanged: same keys, shapes, net_arch [128, 128], Box vs MultiDiscrete heads"""
    meta = json.load(open(os.path.join(GOLD, "policy_meta.json")))[run]
    sd = {k: torch.as_tensor(v) for k, v in np.load(os.path.join(GOLD, f"policy_{run}.npz")).items()}
    A, K = meta["num_arms"], meta["max_num_objects"]
    toggle = meta["env_class"].endswith("ToggleEnv")
    obs_dim = 24 * A + 13 * K + (8 * A if toggle else 0)
    pol = (ActorCriticPolicy(obs_dim, nvec=[2] * A, net_arch=meta["net_arch"]) if toggle else
           ActorCriticPolicy(obs_dim, action_dim=8 * A, net_arch=meta["net_arch"]))
    assert set(pol.state_dict()) == set(sd)
    pol.load_state_dict(sd)
    obs = torch.randn(32, obs_dim)
    a, v, lp = pol(obs)
    assert a.shape == (32, A if toggle else 8 * A) and v.shape == (32,) and torch.isfinite(lp).all()
    v2, lp2, ent = pol.evaluate_actions(obs, a)
    torch.testing.assert_close(v2, v)
    torch.testing.assert_close(lp2, lp)
    # the MLP forward is the definition (Linear -> Tanh -> Linear -> Tanh -> heads)
    h = torch.tanh(obs @ sd["mlp_extractor.policy_net.0.weight"].T + sd["mlp_extractor.policy_net.0.bias"])
    h = torch.tanh(h @ sd["mlp_extractor.policy_net.2.weight"].T + sd["mlp_extractor.policy_net.2.bias"])
    head = h @ sd["action_net.weight"].T + sd["action_net.bias"]
    det = pol.predict(obs, deterministic=True)
    if toggle:
        torch.testing.assert_close(det, head.view(32, A, 2).argmax(-1).float())
    else:
        torch.testing.assert_close(det, head)


def test_gae_matches_rollout_buffer_restatement():
    rng = np.random.default_rng(0)
    T, N = 12, 7
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    st = (rng.random((T, N)) < 0.2).astype(np.float32)
    lv = rng.normal(size=N).astype(np.float32)
    ls = (rng.random(N) < 0.3).astype(np.float32)
    adv, ret = compute_gae(*(torch.as_tensor(x) for x in (r, v, st, lv, ls)), 0.99, 0.95)
    adv_ref, ret_ref = gae_reference(r.astype(np.float64), v.astype(np.float64), st, lv.astype(np.float64), ls, 0.99,
                                     0.95)
    np.testing.assert_allclose(adv.numpy(), adv_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret.numpy(), ret_ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("discrete", [False, True])
def test_ppo_learns_toy_env(discrete, tmp_path):
    env = ToyEnv(n=64, discrete=discrete)
    ppo = PPO(env, policy_kwargs=dict(net_arch=(32, 32)), n_steps=16, batch_size=256, n_epochs=4,
              learning_rate=3e-3, seed=1)
    ppo.learn(64 * 16 * 25)
    first, last = ppo.logs[0]["reward_per_step"], ppo.logs[-1]["reward_per_step"]
    assert last > first + 0.3 * abs(first), (first, last)
    p = str(tmp_path / "ckpt.zip")
    ppo.save(p)
    ppo2 = PPO(ToyEnv(n=8, discrete=discrete), policy_kwargs=dict(net_arch=(32, 32)), seed=5).load_policy(p)
    for a, b in zip(ppo.policy.state_dict().values(), ppo2.policy.state_dict().values()):
        torch.testing.assert_close(a, b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different init per rank: the trainer must broadcast rank 0's weights
    env = ToyEnv(n=32, seed=rank)  # different arenas per rank
    ppo = PPO(env, policy_kwargs=dict(net_arch=(16, 16)), n_steps=8, batch_size=64, n_epochs=2, seed=3, dist=dist)
    t = [torch.tensor([float(rank + 1), 2.0 * rank])]
    flat_allreduce(t, dist)
    ppo.learn(32 * 8 * world * 3)
    params = torch.cat([p.detach().reshape(-1) for p in ppo.policy.parameters()])
    q.put((rank, t[0].tolist(), params.numpy(), ppo.num_timesteps, ppo.logs[-1]["episodes"]))
    dist.destroy_process_group()


def test_data_parallel_ppo_gloo_world2():
    """two ranks with different arenas: the fused all-reduces keep the replicas bit-identical, the advantage
    statistics and episode counts are global"""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert out[0][1] == out[1][1] == [3.0, 2.0]
    np.testing.assert_array_equal(out[0][2], out[1][2])
    assert out[0][3] == out[1][3] == 32 * 8 * 2 * 3
    assert out[0][4] == out[1][4] == 2 * 32  # episodes of 8 steps: every arena of both ranks ended once


def _identical_arenas_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = ToyEnv(n=16, seed=0)  # the SAME arenas on both ranks (bench / FactoryVecEnv default: seed 42 everywhere)
    ppo = PPO(env, policy_kwargs=dict(net_arch=(16, 16)), n_steps=4, batch_size=32, n_epochs=1, seed=3, dist=dist)
    buf, _ = ppo.collect_rollouts()
    q.put((rank, buf["actions"].numpy()))
    dist.destroy_process_group()


def test_ranks_sample_different_actions_on_identical_arenas():
    """data-parallel ranks with identical arenas and broadcast weights still draw independent actions (a per-rank
    sampling stream): their rollouts differ, so the global batch holds world x independent samples"""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_identical_arenas_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    a0, a1 = out[0][1], out[1][1]
    assert a0.shape == a1.shape
    assert not np.array_equal(a0, a1)
