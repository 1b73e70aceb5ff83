"""Policy fixtures from the reference's own checkpoints (runs/*.zip, stable-baselines3 2.3.2 saves).

Only policy.pth (a torch state_dict) is read, with torch.load(weights_only=True) -- nothing in the
archive is executed.  All four runs are kept as float32 .npz data, e.g. rk5rxnav (AllFullRLProgressRewardEnv,
2 arms x 10 cubes, Box(16) actions, obs 178) and y6lp1j7k (PauseIKToggleEnv, 4 arms x 10 cubes,
MultiDiscrete([2]*4), obs 258).  Usage: python tests/golden/gen_policy_fixtures.py
"""
import io
import json
import os
import zipfile

import numpy as np
import torch

REF = "/root/reference/runs"
OUT = os.path.dirname(os.path.abspath(__file__))

if __name__ == "__main__":
    meta = {}
    for run in ["rk5rxnav", "r666unuv", "xfwgqibb", "y6lp1j7k"]:
        with zipfile.ZipFile(os.path.join(REF, f"{run}.zip")) as z:
            sd = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True, map_location="cpu")
        cfg = json.load(open(os.path.join(REF, f"{run}.json")))
        np.savez_compressed(os.path.join(OUT, f"policy_{run}.npz"),
                            **{k: v.numpy().astype(np.float32) for k, v in sd.items()})
        meta[run] = dict(env_class=cfg["env_class"], num_arms=cfg["env_kwargs"]["num_arms"],
                         max_num_objects=cfg["env_kwargs"]["max_num_objects"], net_arch=cfg["policy_kwargs"]["net_arch"],
                         gamma=cfg["gamma"], n_steps=cfg["n_steps"], batch_size=cfg["batch_size"],
                         learning_rate=cfg["learning_rate"], n_epochs=cfg["n_epochs"], ent_coef=cfg["ent_coef"],
                         vf_coef=cfg["vf_coef"], max_grad_norm=cfg["max_grad_norm"], gae_lambda=cfg["gae_lambda"],
                         env_kwargs=cfg["env_kwargs"])
    json.dump(meta, open(os.path.join(OUT, "policy_meta.json"), "w"), indent=1)
    print(json.dumps(meta, indent=1)[:800])
