#!/usr/bin/env python3
"""Fixtures from the reference's own MuJoCo runs (TEST INFRASTRUCTURE; run in the container, never at test time).

The four saved PPO runs (``/root/reference/runs/*.zip``, SB3 2.3.2 checkpoints) hold the only MuJoCo-produced
numbers in the reference: ``_last_obs`` -- the last observation of each of the 8 SubprocVecEnv workers when
training stopped (float32 for the full-joint-control classes, float64 for the toggle classes, whose IK proposals
are float64, environments.py:576) -- and ``ep_info_buffer``, the Monitor ``{"r", "l", "t"}`` records of the last
100 episodes.  They are decoded with sb3_reader.py (a pickletools opcode walk; nothing is unpickled) and written
as plain arrays:

    tests/golden/runs_fixtures.npz   last_obs_<run> [8, obs_dim], ep_r_<run>, ep_l_<run> [100]
    tests/golden/runs_fixtures.json  per run: env_class, env_kwargs, n_envs, num_timesteps, obs dtype

usage: python tests/golden/gen_run_fixtures.py [/root/reference/runs]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import sb3_reader  # noqa: E402

RUNS = ["rk5rxnav", "r666unuv", "xfwgqibb", "y6lp1j7k"]


def main(src="/root/reference/runs"):
    arrays, meta = {}, {}
    for run in RUNS:
        plain, dec = sb3_reader.read_run(os.path.join(src, f"{run}.zip"))
        cfg = json.load(open(os.path.join(src, f"{run}.json")))
        lo = dec["_last_obs"]
        ep = dec["ep_info_buffer"]
        arrays[f"last_obs_{run}"] = lo
        arrays[f"ep_r_{run}"] = np.array([e["r"] for e in ep], np.float64)
        arrays[f"ep_l_{run}"] = np.array([e["l"] for e in ep], np.int64)
        kw = {k: v for k, v in cfg["env_kwargs"].items() if k != "render_mode"}
        meta[run] = dict(env_class=cfg["env_class"], env_kwargs=kw, n_envs=int(plain["n_envs"]),
                         num_timesteps=int(plain["num_timesteps"]), obs_dtype=str(lo.dtype),
                         last_episode_starts=[bool(x) for x in dec["_last_episode_starts"]],
                         source=f"runs/{run}.zip data: _last_obs, ep_info_buffer (SB3 2.3.2)")
    np.savez_compressed(os.path.join(HERE, "runs_fixtures.npz"), **arrays)
    with open(os.path.join(HERE, "runs_fixtures.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote runs_fixtures.npz / .json:", {k: v.shape for k, v in arrays.items() if k.startswith("last_obs")})


if __name__ == "__main__":
    main(*sys.argv[1:])
