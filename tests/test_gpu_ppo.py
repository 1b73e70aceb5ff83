"""PPO on the GPU env (factory_marl_amd/ppo.py over FactoryVecEnv) and the reference's trained policies
(runs/*.zip policy.pth, kept as fixtures) driving our HIP env."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _have_gpu():
    return torch.cuda.is_available()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_ppo_iterations_on_gpu_env():
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs
    from factory_marl_amd.ppo import PPO

    env = FactoryVecEnv(512, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42))
    ppo = PPO(env, n_steps=8, batch_size=1024, n_epochs=2, seed=0)
    ppo.learn(512 * 8 * 2)
    assert ppo.num_timesteps == 512 * 8 * 2 and len(ppo.logs) == 2
    for rec in ppo.logs:
        assert all(np.isfinite(rec[k]) for k in ["policy_loss", "value_loss", "entropy_loss", "reward_per_step"])
    env.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
@pytest.mark.parametrize("run", ["rk5rxnav", "y6lp1j7k"])
def test_reference_policy_drives_gpu_env(run):
    """the reference's trained SB3 policy, loaded unchanged, drives 256 arenas of the matching env class on the
    GPU (deterministic actions): finite observations, episodes end and restart, no contact-capacity drops"""
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.ppo import ActorCriticPolicy

    meta = json.load(open(os.path.join(GOLD, "policy_meta.json")))[run]
    kw = {k: v for k, v in meta["env_kwargs"].items() if k != "render_mode"}
    env = FactoryVecEnv(256, env_class=meta["env_class"], env_kwargs=kw)
    pol = ActorCriticPolicy.for_env(env, net_arch=meta["net_arch"]).to(env.device)
    sd = {k: torch.as_tensor(v) for k, v in np.load(os.path.join(GOLD, f"policy_{run}.npz")).items()}
    pol.load_state_dict(sd)
    env.reset()
    obs = env.obs.clone()
    ret = torch.zeros(256, device=env.device)
    ended = 0
    scores = []
    for _ in range(150):
        a = pol.predict(obs, deterministic=True)
        if not pol.discrete:
            a = a.clamp(-1, 1)
        o, r, term, _ = env.step_tensors(a.contiguous())
        ret += r
        ended += int(term.sum())
        if term.any():
            scores.append(env.terminal_scores[term.bool()].sum(1).float().mean().item())
        obs = o.clone()
    env.sync()
    cnt = env.counters()
    print(f"{run} ({meta['env_class']} {kw['num_arms']}x{kw['max_num_objects']}): mean return over 150 steps "
          f"{ret.mean().item():.3f}, episodes ended {ended}, mean terminal score {np.mean(scores) if scores else 0:.2f}, "
          f"contacts dropped {int(cnt[:, 0].sum())}, max contacts {int(cnt[:, 5].max())}")
    assert torch.isfinite(obs).all() and torch.isfinite(ret).all()
    env.close()


@pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")
def test_rccl_collectives_execute_on_the_gpu():
    """the trainer's RCCL path on hardware (backend "nccl" = RCCL on ROCm), one rank on the box's one GPU: the process
    group opened as launch.RankContext opens it for GPU ranks, a device all-reduce, and one PPO iteration with the
    group live -- initial-weight broadcast, the asynchronous advantage-statistics all-reduce and the fused gradient
    all-reduce (ppo.py) all go through RCCL kernels.  (The 8-GPU node is the driver's; world 1 exercises the calls.)"""
    import socket

    import torch.distributed as dist

    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs
    from factory_marl_amd.launch import reduce_over_ranks
    from factory_marl_amd.ppo import PPO

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        t = torch.arange(16, dtype=torch.float32, device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        assert torch.equal(t, torch.arange(16, dtype=torch.float32, device=dev))
        assert reduce_over_ranks(2.5, "max", dev) == 2.5
        env = FactoryVecEnv(256, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4,
                                                        seed=42))
        ppo = PPO(env, n_steps=4, batch_size=512, n_epochs=1, seed=0, dist=dist)
        assert ppo.dist is not None and ppo.world == 1
        ppo.learn(256 * 4)
        rec = ppo.logs[-1]
        assert all(np.isfinite(rec[k]) for k in ["policy_loss", "value_loss", "entropy_loss"])
        env.close()
    finally:
        dist.destroy_process_group()
