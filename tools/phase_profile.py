"""Phase profile of the env-step kernel (fm_profile): where the wall time of one env-step goes.

Usage (GPU box): python tools/phase_profile.py [--arenas 4096] [--steps 10] [--precision fp32]
Times are wall-clock ticks summed over arenas, so they are reported as a share of the total and as
microseconds per arena-substep.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root (bench, package)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arenas", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--arms", type=int, default=2)
    ap.add_argument("--objects", type=int, default=4)
    ap.add_argument("--preroll", type=int, default=200, help="desynchronising pre-roll (bench.preroll)")
    ap.add_argument("--env-class", default="AllFullRLProgressRewardEnv")
    args = ap.parse_args()
    import torch

    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    env = FactoryVecEnv(args.arenas, env_class=args.env_class,
                        env_kwargs=run_kwargs(args.env_class, num_arms=args.arms, max_num_objects=args.objects, seed=42),
                        precision=args.precision, return_numpy=False)
    toggles = args.env_class in ("PauseIKToggleEnv", "BackupIKToggleEnv")

    def act():
        u = torch.rand(args.arenas, env.act_dim, device=env.device, generator=g)
        return (u < 0.5).float() if toggles else u * 2 - 1

    env.reset()
    import bench

    bench.preroll(env, args.preroll, 0, env.device)
    g = torch.Generator(device=env.device)
    g.manual_seed(0)
    for _ in range(5):
        env.step_tensors(act())
    env.sync()
    c0 = env.counters().sum(0)
    env.profile(1)
    for _ in range(args.steps):
        env.step_tensors(act())
    env.sync()
    ph, ncon = env.profile(0)
    c1 = env.counters().sum(0)
    if args.arms * 9 + args.objects * 6 + 1 <= 80:  # no dense Cholesky: its slots carry the narrowphase split
        for a, b in (("chol_diag", "coll_narrow_expand"), ("chol_panel", "coll_narrow_other"),
                     ("chol_trail", "coll_narrow_boxbox")):
            ph[b] = ph.pop(a)
        ph["coll_narrow"] = ph["coll_narrow"] + ph["coll_narrow_expand"] + ph["coll_narrow_other"] + ph["coll_narrow_boxbox"]
        narrow_split = ("coll_narrow_expand", "coll_narrow_other", "coll_narrow_boxbox")
    else:
        narrow_split = ()
    tot = sum(v for k, v in ph.items() if k not in narrow_split)
    sub = args.arenas * args.steps * 100
    rep = {k: {"share": round(v / tot, 4), "us_per_arena_substep": round(v / sub * 1e6, 3)} for k, v in ph.items()}
    rep["_total_us_per_arena_substep"] = round(tot / sub * 1e6, 3)
    coll = sum(ph[k] for k in ("coll_bounds", "coll_midphase", "coll_narrow", "collision"))
    rep["_collision_total_us_per_arena_substep"] = round(coll / sub * 1e6, 3)  # "collision" = the contact ranking
    chol = sum(ph.get(k, 0.0) for k in ("newton_chol", "chol_diag", "chol_panel", "chol_trail", "chol_solve"))
    rep["_cholesky_total_us_per_arena_substep"] = round(chol / sub * 1e6, 3)
    rep["_mean_ncon"] = round(ncon / sub, 3)
    rep["_lds_bytes_per_arena"] = env._L.fm_workspace_bytes(env._h)
    rep["_newton_iters_per_substep"] = round(float(c1[1] - c0[1]) / sub, 3)
    rep["_mean_objects_in_scene"] = round(float(c1[6] - c0[6]) / (args.arenas * args.steps), 3)
    rep["_preroll"] = args.preroll
    rep["_scene"] = f"{args.arms}x{args.objects}"
    rep["_env_class"] = args.env_class
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
