"""Debug driver (GPU box): teacher-forced comparison of the HIP env-step against the oracle, verbose."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import pyoracle as po  # noqa: E402  (test infrastructure: checker only)
from factory_marl_amd import FactoryVecEnv, state as st  # noqa: E402

A, K = 2, 4
prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
po.build()
rng = np.random.default_rng(7)
e = po.Env(A, K, 42, reward="progress", weights=(0.2, 0.4, 0.1, 0.4))
ref0 = e.reset()
env = FactoryVecEnv(1, env_kwargs=dict(num_arms=A, max_num_objects=K, seed=42, gripper_to_closest_cube_reward_factor=0.2,
                                     closest_cube_to_bucket_reward_factor=0.4, small_action_norm_reward_factor=0.1,
                                     base_reward=0.4),
                    precision=prec)
obs = env.reset()
torch.cuda.synchronize()
print("reset obs max diff", np.abs(np.asarray(obs)[0] - ref0).max(), flush=True)
nq, nv, nu, nd, ni = st.sizes(A, K)
g0 = st.unpack(A, K, env.get_state()[0])
d0, i0, r0 = e.export_state()
print("reset state diff dbl", np.abs(g0[0] - d0).max(), "ints eq", np.array_equal(g0[1], i0), "rng eq",
      np.array_equal(g0[2], r0), flush=True)
fd = st.fields(A, K, g0[0])
fo = st.fields(A, K, d0)
for k in fd:
    print("  ", k, np.abs(fd[k] - fo[k]).max())
for t in range(int(sys.argv[2]) if len(sys.argv) > 2 else 30):
    d, i, r = e.export_state()
    rec = st.pack(A, K, d, i, r)
    env.set_state(rec[None])
    a = rng.uniform(-2, 2, 8 * A).astype(np.float32)
    t0 = time.time()
    gobs, grew, gterm, _ = env.step_tensors(torch.as_tensor(a[None], device=env.device))
    env.sync()
    dt = time.time() - t0
    obs, rew, term, _, info = e.step(a)
    gd, gi, gr = st.unpack(A, K, env.get_state()[0])
    od, oi, orng = e.export_state()
    fg, fo = st.fields(A, K, gd), st.fields(A, K, od)
    errs = {k: float(np.abs(fg[k] - fo[k]).max()) for k in ["qpos", "qvel", "qacc_warmstart", "ctrl_target"]}
    print(f"t={t} term ref={term} gpu={bool(gterm.item())} rew ref={rew:.6f} gpu={grew.item():.6f} "
          f"ints_eq={np.array_equal(gi, oi)} rng_eq={np.array_equal(gr, orng)} errs={errs} "
          f"ncon_ref={e.data.ncon} iters_ref={e.data.niter} gpu_ms={dt*1e3:.1f} ctr={env.counters()[0]}",
          flush=True)
    if errs["qpos"] > 1e-3:
        qd = np.abs(fg["qpos"] - fo["qpos"])
        vd = np.abs(fg["qvel"] - fo["qvel"])
        print("   qpos worst idx", np.argsort(-qd)[:6], qd[np.argsort(-qd)[:6]])
        print("   qvel worst idx", np.argsort(-vd)[:6], vd[np.argsort(-vd)[:6]])
        print("   gpu qpos", np.round(fg["qpos"], 5))
        print("   ref qpos", np.round(fo["qpos"], 5))
    if term:
        e.reset()
        env.reset()
