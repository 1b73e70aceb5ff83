"""Probe: teacher-forced batch vs. single-arena results of the same oracle states (interference check)."""
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
    for t in range(96):
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

    def run(idx):
        env = FactoryVecEnv(len(idx), env_kwargs=kw, precision=prec)
        env.reset()
        env.set_state(recs[idx])
        env.step_tensors(torch.as_tensor(acts[idx], device=env.device))
        env.sync()
        out = env.get_state()
        env.close()
        return out

    full = run(np.arange(96))
    full2 = run(np.arange(96))
    print("batch run-to-run identical:", np.array_equal(full, full2))
    for s in [4, 5, 48, 93]:
        one = run(np.array([s]))
        four = run(np.array([s, 0, 1, 2]))
        print(f"state {s}: batch==single {np.array_equal(full[s], one[0])}, batch==4-batch {np.array_equal(full[s], four[0])}, "
              f"single==4 {np.array_equal(one[0], four[0])}")
        nq, nv = st.sizes(A, K)[:2]
        d1 = st.unpack(A, K, full[s])[0]
        d2 = st.unpack(A, K, one[0])[0]
        print("   max |qvel batch - single|", np.abs(d1[nq:nq + nv] - d2[nq:nq + nv]).max())


if __name__ == "__main__":
    main()
