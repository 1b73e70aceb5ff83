#!/usr/bin/env python3
"""Behavioural statistics of the GPU env against the reference's own MuJoCo numbers (test infrastructure).

* IK base policy (FactoryManipulationEnv, every arm on the IK policy): report/report.tex:276-295 gives, over 100
  episodes of one env (visualisation.py:55-85: sequential episodes, the TaskManager RNG running on; length = the
  0-based index t of the terminating step), (1.65, 1.17) / 208.8 for 2 arms and (1.18, 1.16) / 119.74 for 4 arms.
  Measured here two ways: the reference protocol (one arena, seed 42, E sequential episodes) and a large sample
  (N arenas with seeds 42 + i, the first episode of each).
* The saved policies (runs/*.zip policy.pth as tests/golden/policy_<run>.npz): SB3 predict() is stochastic by
  default (Gaussian / categorical sampling), the runs' ep_info_buffer holds the Monitor (r, l) of their last 100
  training episodes (tests/golden/runs_fixtures.npz).

usage: python tools/behaviour.py base A [--arenas N] [--episodes E] [--precision fp64]
       python tools/behaviour.py policy RUN [--arenas N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")


def _stats(x):
    x = np.asarray(x, np.float64)
    return dict(mean=float(x.mean()), se=float(x.std(ddof=1) / np.sqrt(len(x))) if len(x) > 1 else 0.0, n=int(len(x)))


def run_episodes(env, act_fn, want_per_arena, max_steps):
    """step until every arena has finished `want_per_arena` episodes; returns per-episode (scores, length, return)"""
    import torch

    N = env.num_envs
    done_count = np.zeros(N, np.int64)
    eps = []
    obs = env.obs
    for step in range(max_steps):
        a = act_fn(obs)
        obs, rew, term, _ = env.step_tensors(a)
        t = term.bool()
        if bool(t.any()):
            idx = torch.nonzero(t).flatten().cpu().numpy()
            sc = env.terminal_scores[idx].cpu().numpy()
            ln = env.ep_len[idx].cpu().numpy()
            rt = env.ep_return[idx].cpu().numpy()
            for j, i in enumerate(idx):
                if done_count[i] < want_per_arena:
                    eps.append((sc[j].tolist(), int(ln[j]), float(rt[j])))
                done_count[i] += 1
        if (done_count >= want_per_arena).all():
            break
        if step % 50 == 49:  # progress on stderr (a long run otherwise looks hung)
            print(f"step {step + 1}: {int((done_count >= want_per_arena).sum())}/{N} arenas done", file=sys.stderr,
                  flush=True)
    return eps, int(step + 1), int((done_count >= want_per_arena).sum())


def sequential_episodes(env, episodes, chunk=2000, max_steps=200_000):
    """the report's protocol on arena 0 (visualisation.py:55-80: env.reset() after each termination -- here the
    kernel's auto-reset, which is reset_sim with the TaskManager RNG running on): per-step flags, terminal scores and
    episode lengths are gathered on the device and read once per chunk (no host sync per env-step); returns the first
    `episodes` episodes as (scores, length, return)"""
    import torch

    dev = env.device
    a = torch.zeros(env.num_envs, env.act_dim, device=dev)  # FactoryManipulationEnv: no action entries
    eps = []
    done = 0
    while len(eps) < episodes and done < max_steps:
        term_h = torch.zeros(chunk, dtype=torch.bool, device=dev)
        sc_h = torch.zeros(chunk, 2, dtype=torch.int32, device=dev)
        len_h = torch.zeros(chunk, dtype=torch.int32, device=dev)
        ret_h = torch.zeros(chunk, dtype=torch.float32, device=dev)
        for t in range(chunk):
            _, _, term, _ = env.step_tensors(a)
            term_h[t] = term[0].bool()
            sc_h[t] = env.terminal_scores[0]
            len_h[t] = env.ep_len[0]
            ret_h[t] = env.ep_return[0]
        done += chunk
        idx = torch.nonzero(term_h).flatten().cpu().numpy()
        sc, ln, rt = sc_h.cpu().numpy(), len_h.cpu().numpy(), ret_h.cpu().numpy()
        eps += [(sc[i].tolist(), int(ln[i]), float(rt[i])) for i in idx]
        print(f"{done} env-steps: {len(eps)} episodes", file=sys.stderr, flush=True)
    return eps[:episodes], done


def base(args):
    import torch

    from factory_marl_amd import FactoryVecEnv

    A = args.A
    out = {}
    kw = dict(num_arms=A, max_num_objects=10, seed=42)
    zero = lambda o: torch.zeros(1, device=o.device)  # noqa: E731  (act_dim 0)
    # the reference protocol: one env, seed 42, sequential episodes
    if args.episodes > 0:
        env = FactoryVecEnv(1, env_class="FactoryManipulationEnv", env_kwargs=kw, precision=args.precision,
                            return_numpy=False)
        env.reset()
        t0 = time.time()
        eps, steps = sequential_episodes(env, args.episodes)
        env.close()
        out["sequential"] = dict(scores0=_stats([e[0][0] for e in eps]), scores1=_stats([e[0][1] for e in eps]),
                                 length_t=_stats([e[1] - 1 for e in eps]), episodes=len(eps),
                                 seconds=time.time() - t0)
    # the large sample: seeds 42 + i, first episode of each arena
    if args.arenas:
        env = FactoryVecEnv(args.arenas, env_class="FactoryManipulationEnv", env_kwargs=kw, precision=args.precision,
                            seeds=42 + np.arange(args.arenas), return_numpy=False)
        env.reset()
        t0 = time.time()
        eps, steps, fin = run_episodes(env, lambda o: torch.zeros(args.arenas, 1, device=o.device), 1, 1500)
        env.close()
        out["parallel"] = dict(scores0=_stats([e[0][0] for e in eps]), scores1=_stats([e[0][1] for e in eps]),
                               length_t=_stats([e[1] - 1 for e in eps]), episodes=len(eps), finished=fin,
                               steps=steps, seconds=time.time() - t0)
    ref = {2: dict(scores=(1.65, 1.17), length=208.8), 4: dict(scores=(1.18, 1.16), length=119.74)}[A]
    out.update(mode="base", A=A, precision=args.precision, reference_report=ref)
    return out


def policy(args):
    import torch

    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.ppo import ActorCriticPolicy

    meta = json.load(open(os.path.join(GOLD, "policy_meta.json")))[args.run]
    kw = {k: v for k, v in meta["env_kwargs"].items() if k != "render_mode"}
    env = FactoryVecEnv(args.arenas, env_class=meta["env_class"], env_kwargs=kw, precision=args.precision,
                        seeds=42 + np.arange(args.arenas) if args.seeds == "arena" else None, return_numpy=False)
    pol = ActorCriticPolicy.for_env(env, net_arch=meta["net_arch"]).to(env.device)
    sd = {k: torch.as_tensor(v) for k, v in np.load(os.path.join(GOLD, f"policy_{args.run}.npz")).items()}
    pol.load_state_dict(sd)
    gen = torch.Generator(device=env.device)
    gen.manual_seed(0)
    env.reset()

    def act(o):
        a = pol.predict(o, deterministic=False, generator=gen)
        return a if pol.discrete else a.clamp(-1.0, 1.0)

    t0 = time.time()
    eps, steps, fin = run_episodes(env, act, 1, 1500)
    env.close()
    z = np.load(os.path.join(GOLD, "runs_fixtures.npz"))
    return dict(mode="policy", run=args.run, env_class=meta["env_class"], precision=args.precision,
                r=_stats([e[2] for e in eps]), l=_stats([e[1] for e in eps]),
                scores0=_stats([e[0][0] for e in eps]), scores1=_stats([e[0][1] for e in eps]), finished=fin,
                steps=steps, seconds=time.time() - t0,
                reference_ep_info=dict(r=_stats(z[f"ep_r_{args.run}"]), l=_stats(z[f"ep_l_{args.run}"])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["base", "policy"])
    ap.add_argument("what")
    ap.add_argument("--arenas", type=int, default=1000)
    ap.add_argument("--episodes", type=int, default=100)
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--seeds", default="arena", choices=["arena", "fixed"])
    args = ap.parse_args()
    if args.mode == "base":
        args.A = int(args.what)
        print(json.dumps(base(args)), flush=True)
    else:
        args.run = args.what
        print(json.dumps(policy(args)), flush=True)


if __name__ == "__main__":
    main()
