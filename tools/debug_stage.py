"""Debug driver (GPU box): compare one recomputed physics stage of the HIP kernel with the oracle."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import pyoracle as po  # noqa: E402  (test infrastructure: checker only)
from factory_marl_amd import FactoryVecEnv, state as st  # noqa: E402
from factory_marl_amd.environments import run_kwargs  # noqa: E402

A, K = 2, 4
prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
po.build()
L = po.lib()
e = po.Env(A, K, 42)
e.reset()
rng = np.random.default_rng(3)
for t in range(nsteps):
    e.step(rng.uniform(-2, 2, 8 * A).astype(np.float32))
env = FactoryVecEnv(1, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=A, max_num_objects=K, seed=42), precision=prec)
env.reset()
d, i, r = e.export_state()
env.set_state(st.pack(A, K, d, i, r)[None])
act = 0 if nsteps == 0 else 1
g = env.debug_dump(0, actuated=bool(act))
# oracle: recompute the same stage (qpos_stage) + forward
m, dd = e.model, e.data
f = st.fields(A, K, d)
dd.qpos[:] = f["qpos_stage"]
dd.qvel[:] = f["qvel_stage"]
dd.qacc_warmstart[:] = f["qacc_warmstart"]
dd.ctrl[:] = f["ctrl_target"]
L.or_d_stage_fwd(m.h, dd.h, act)
nv = m.nv
a0 = 1 + 6 * K
M = dd.M
for arm in range(A):
    Mo = M[a0 + 9 * arm:a0 + 9 * arm + 9, a0 + 9 * arm:a0 + 9 * arm + 9]
    Mg = g["Marm"][81 * arm:81 * arm + 81].reshape(9, 9)
    print(f"arm{arm} M maxdiff", np.abs(Mo - Mg).max(), "rel", np.abs(Mo - Mg).max() / np.abs(Mo).max())
    if arm == 0:
        np.set_printoptions(linewidth=200, precision=6, suppress=True)
        print("Mref\n", Mo)
        print("Mgpu\n", Mg)
qp = np.ctypeslib.as_array(L.or_d_qfrc_passive(dd.h), shape=(nv,))
pb_o = qp - dd.qfrc_bias
print("pb maxdiff", np.abs(pb_o - g["pb"]).max(), "idx", np.argsort(-np.abs(pb_o - g["pb"]))[:5])
print("  pb ref", np.round(pb_o[a0:], 5))
print("  pb gpu", np.round(g["pb"][a0:], 5))
qs = np.ctypeslib.as_array(L.or_d_qacc_smooth(dd.h), shape=(nv,))
print("qacc_smooth maxdiff", np.abs(qs - g["as"]).max(), "idx", np.argsort(-np.abs(qs - g["as"]))[:5])
print("qacc maxdiff", np.abs(dd.qacc - g["a"]).max(), "idx", np.argsort(-np.abs(dd.qacc - g["a"]))[:5])
print("  qacc ref", np.round(dd.qacc[a0:], 4))
print("  qacc gpu", np.round(g["a"][a0:], 4))
print("qfrc_constraint maxdiff", np.abs(dd.qfrc_constraint - g["fc"]).max())
print("ncon ref", dd.ncon, "gpu", g["ncon"], "nefc ref", dd.nefc, "gpu rows", g["nrow"])
cons = dd.contacts()
for c in cons[:20]:
    print("  ref con", c["geom"], round(c["dist"], 6), np.round(c["pos"], 4), np.round(c["frame"][0], 3), c["mu"])
for c in g["con"][:20]:
    print("  gpu con", (int(c[0]), int(c[1])), round(c[2], 6), np.round(c[3:6], 4), np.round(c[6:9], 3), c[15])
# bodies: oracle xpos of arm0 links
bo = 16 + K + 14 * 0
print("xipos ref arm0 bodies", np.round(dd.xipos[bo + 3:bo + 14], 5).tolist())
print("bcom gpu arm0", np.round(g["bcom"][:30].reshape(10, 3), 5).tolist())
print("xpos ref arm0 all", np.round(dd.xpos[bo + 3:bo + 14], 5).tolist())
print("bpos gpu arm0 all", np.round(g["bpos"][:30].reshape(10, 3), 5).tolist())
print("xpos ref arm0 links", np.round(dd.xpos[bo + 3:bo + 10], 4).tolist())
print("xpos gpu arm0 links", np.round(g["bpos"][:21].reshape(7, 3), 4).tolist())
print("site ref", np.round(dd.site_xpos, 5).tolist(), "gpu", np.round(g["site"], 5).tolist())
print("rows gpu", np.round(g["rows"], 5).tolist())
