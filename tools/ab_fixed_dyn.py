"""A/B: the compile-time-specialised env-step kernel vs the runtime-dims kernel on identical states."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from factory_marl_amd import FactoryVecEnv, state as st
    from oracle import pyoracle

    A, K = 2, 4
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
    pyoracle.build()
    e = pyoracle.Env(A, K, 42, reward="progress", weights=(0.2, 0.4, 0.1, 0.4))
    e.reset()
    rng = np.random.default_rng(7)
    recs, acts = [], []
    for t in range(12):
        d, i, r = e.export_state()
        recs.append(st.pack(A, K, d, i, r))
        a = rng.uniform(-2, 2, 8 * A).astype(np.float32)
        acts.append(a)
        _, _, term, _, _ = e.step(a)
        if term:
            e.reset()
    recs, acts = np.stack(recs), np.stack(acts)
    kw = dict(num_arms=A, max_num_objects=K, seed=42, gripper_to_closest_cube_reward_factor=0.2,
              closest_cube_to_bucket_reward_factor=0.4, small_action_norm_reward_factor=0.1, base_reward=0.4)
    outs = {}
    for mode in ["dyn", "fixed"]:
        os.environ["FM_FORCE_DYNAMIC"] = "1" if mode == "dyn" else "0"
        env = FactoryVecEnv(len(recs), env_kwargs=kw, precision=prec)
        env.reset()
        env.set_state(recs)
        env.step_tensors(torch.as_tensor(acts, device=env.device))
        env.sync()
        outs[mode] = (env.get_state(), env.counters())
        env.close()
    nq, nv, nu, nd, ni = st.sizes(A, K)
    for s in range(len(recs)):
        gd0, gi0, _ = st.unpack(A, K, outs["dyn"][0][s])
        gd1, gi1, _ = st.unpack(A, K, outs["fixed"][0][s])
        dq = np.abs(gd0[:nq] - gd1[:nq]).max()
        dv = np.abs(gd0[nq:nq + nv] - gd1[nq:nq + nv])
        j = int(np.argmax(dv))
        print(f"step {s}: |dq| {dq:.3e} |dv| {dv.max():.3e} at qvel[{j}] dyn {gd0[nq + j]:.6g} fixed {gd1[nq + j]:.6g} "
              f"ints equal {np.array_equal(gi0, gi1)} ctr dyn {outs['dyn'][1][s]} fixed {outs['fixed'][1][s]}")


if __name__ == "__main__":
    main()
