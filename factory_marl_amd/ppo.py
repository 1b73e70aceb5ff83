"""PPO on the GPU env: the training path of the reference (src/learning.py:20-120) on PyTorch-ROCm.

The reference trains stable-baselines3 PPO ("MlpPolicy", net_arch [128, 128], gamma 0.99, SB3 defaults
otherwise: runs/*.json) over a SubprocVecEnv of CPU MuJoCo arenas.  stable-baselines3 is not installed in
this image, so this module restates the parts of SB3 2.3.2 the reference uses, on device tensors end to end:

* ``ActorCriticPolicy`` -- SB3's MlpPolicy: separate tanh MLPs for policy and value
  (``mlp_extractor.policy_net`` / ``mlp_extractor.value_net``), ``action_net``, ``value_net``, a state-independent
  ``log_std`` for Box actions (DiagGaussian) or per-dimension Categoricals for MultiDiscrete (the IK toggles);
  orthogonal init with SB3's gains.  The ``state_dict`` keys and shapes are SB3's, so the reference's own
  checkpoints (runs/*.zip -> policy.pth) load with ``torch.load(weights_only=True)``.
* ``PPO`` -- SB3's rollout / GAE(lambda) / clipped-surrogate update (n_epochs x shuffled minibatches,
  per-minibatch advantage normalisation, value MSE, entropy bonus, grad-norm clip, Adam eps 1e-5), with the
  rollout buffer, GAE and losses all on the GPU and the env stepped through ``FactoryVecEnv.step_tensors``
  (zero copy).  Box actions are clipped to [-1, 1] before the env sees them and stored unclipped, as SB3 does.
* Data parallel over ranks: every rank owns its own arenas (no env-side exchange).  Per
  minibatch: the advantage statistics (sum, sum of squares, count; 3 floats) are all-reduced asynchronously
  while the forward pass runs, so the normalisation uses the global minibatch as a single-process SB3 run over
  all arenas would; after backward ONE all-reduce over a flat buffer carries every gradient (~0.1 M floats
  for [128, 128]).  Episode statistics are all-reduced once per rollout.  With the "nccl" backend the
  collectives are RCCL over xGMI.

n_steps / batch_size: SB3's 2048 x 64 does not scale to 16k-131k arenas; the caller chooses them (defaults here:
n_steps 16, batch_size 8192 per rank) and they are recorded in ``data`` of every checkpoint.
"""
import io
import json
import math
import time
import zipfile

import numpy as np
import torch
import torch.nn as nn

__all__ = ["ActorCriticPolicy", "PPO", "load_sb3_policy_state", "flat_allreduce", "compute_gae"]


class _MlpExtractor(nn.Module):
    def __init__(self, obs_dim, net_arch):
        super().__init__()

        def mlp():
            layers, last = [], obs_dim
            for h in net_arch:
                layers += [nn.Linear(last, h), nn.Tanh()]
                last = h
            return nn.Sequential(*layers)

        self.policy_net = mlp()
        self.value_net = mlp()
        self.latent_dim = net_arch[-1] if net_arch else obs_dim


class ActorCriticPolicy(nn.Module):
    """SB3 ActorCriticPolicy with the default MlpExtractor (stable_baselines3/common/policies.py)."""

    def __init__(self, obs_dim, action_dim=None, nvec=None, net_arch=(64, 64), log_std_init=0.0, ortho_init=True):
        super().__init__()
        if (action_dim is None) == (nvec is None):
            raise ValueError("give action_dim (Box) or nvec (MultiDiscrete)")
        self.obs_dim = int(obs_dim)
        self.discrete = nvec is not None
        self.nvec = [int(n) for n in nvec] if self.discrete else None
        self.action_dim = len(self.nvec) if self.discrete else int(action_dim)
        self.mlp_extractor = _MlpExtractor(self.obs_dim, list(net_arch))
        lat = self.mlp_extractor.latent_dim
        if self.discrete:
            self.action_net = nn.Linear(lat, sum(self.nvec))
        else:
            self.action_net = nn.Linear(lat, self.action_dim)
            self.log_std = nn.Parameter(torch.ones(self.action_dim) * log_std_init)
        self.value_net = nn.Linear(lat, 1)
        if ortho_init:  # SB3: mlp_extractor sqrt(2), action_net 0.01, value_net 1; biases 0
            for mod, gain in [(self.mlp_extractor, math.sqrt(2)), (self.action_net, 0.01), (self.value_net, 1.0)]:
                for m in mod.modules():
                    if isinstance(m, nn.Linear):
                        nn.init.orthogonal_(m.weight, gain=gain)
                        m.bias.data.fill_(0.0)

    # ------------------------------------------------------------------ distributions
    def _dist_params(self, obs):
        obs = obs.float()  # SB3 preprocess_obs: Box observations as float32 (the toggle envs' rows are float64)
        lp = self.mlp_extractor.policy_net(obs)
        lv = self.mlp_extractor.value_net(obs)
        return self.action_net(lp), self.value_net(lv).squeeze(-1)

    def _log_prob_entropy(self, head, actions):
        if self.discrete:
            lps, ents, o = [], [], 0
            for i, n in enumerate(self.nvec):
                logits = head[:, o:o + n]
                o += n
                logp = torch.log_softmax(logits, dim=-1)
                a = actions[:, i].long()
                lps.append(logp.gather(1, a[:, None]).squeeze(1))
                ents.append(-(logp.exp() * logp).sum(-1))
            return torch.stack(lps, 1).sum(1), torch.stack(ents, 1).sum(1)
        std = self.log_std.exp().expand_as(head)
        var = std * std
        logp = -((actions - head) ** 2) / (2 * var) - self.log_std - math.log(math.sqrt(2 * math.pi))
        ent = 0.5 + 0.5 * math.log(2 * math.pi) + self.log_std
        return logp.sum(-1), ent.expand_as(head).sum(-1)

    def _sample(self, head, deterministic, generator=None):
        """`generator`: the sampling stream (PPO keeps one per rank); None = torch's global RNG"""
        if self.discrete:
            outs, o = [], 0
            for n in self.nvec:
                logits = head[:, o:o + n]
                o += n
                if deterministic:
                    outs.append(logits.argmax(-1))
                else:
                    outs.append(torch.multinomial(torch.softmax(logits, -1), 1, generator=generator).squeeze(1))
            return torch.stack(outs, 1).to(torch.float32)
        if deterministic:
            return head
        noise = torch.randn(head.shape, device=head.device, dtype=head.dtype, generator=generator)
        return head + self.log_std.exp() * noise

    # ------------------------------------------------------------------ SB3 API
    def forward(self, obs, deterministic=False, generator=None):
        head, values = self._dist_params(obs)
        actions = self._sample(head, deterministic, generator)
        logp, _ = self._log_prob_entropy(head, actions)
        return actions, values, logp

    def evaluate_actions(self, obs, actions):
        head, values = self._dist_params(obs)
        logp, ent = self._log_prob_entropy(head, actions)
        return values, logp, ent

    def predict_values(self, obs):
        obs = obs.float()
        return self.value_net(self.mlp_extractor.value_net(obs)).squeeze(-1)

    @torch.no_grad()
    def predict(self, obs, deterministic=True, generator=None):
        head, _ = self._dist_params(obs)
        return self._sample(head, deterministic, generator)

    @classmethod
    def for_env(cls, env, net_arch=(128, 128), **kw):
        sp = env.action_space
        if hasattr(sp, "nvec"):
            return cls(env.obs_dim, nvec=list(sp.nvec), net_arch=net_arch, **kw)
        return cls(env.obs_dim, action_dim=env.act_dim, net_arch=net_arch, **kw)


def load_sb3_policy_state(path):
    """state_dict of an SB3 checkpoint zip (policy.pth) with a loader that executes nothing from the file"""
    with zipfile.ZipFile(path) as z:
        return torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True, map_location="cpu")


def flat_allreduce(tensors, dist, group=None):
    """one all-reduce (sum) over a list of tensors packed into a single flat buffer; results written back"""
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, group=group)
    o = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[o:o + n].view_as(t))
        o += n
    return tensors


class PPO:
    """SB3 PPO (stable_baselines3/ppo/ppo.py) over a FactoryVecEnv; hyperparameters default to SB3's, except
    n_steps / batch_size (see module docstring)."""

    def __init__(self, env, policy_kwargs=None, learning_rate=3e-4, n_steps=16, batch_size=8192, n_epochs=10,
                 gamma=0.99, gae_lambda=0.95, clip_range=0.2, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
                 normalize_advantage=True, seed=0, dist=None, policy=None):
        self.env = env
        self.device = env.device
        self.dist = dist if (dist is not None and dist.is_available() and dist.is_initialized()) else None
        self.world = self.dist.get_world_size() if self.dist else 1
        pk = dict(net_arch=(128, 128))
        pk.update(policy_kwargs or {})
        torch.manual_seed(seed)
        self.policy = (policy or ActorCriticPolicy.for_env(env, **pk)).to(self.device)
        if self.dist:  # identical initial weights on every rank
            for p in self.policy.parameters():
                self.dist.broadcast(p.data, 0)
        self.optimizer = torch.optim.Adam(self.policy.parameters(), lr=learning_rate, eps=1e-5)
        self.hp = dict(learning_rate=learning_rate, n_steps=n_steps, batch_size=batch_size, n_epochs=n_epochs,
                       gamma=gamma, gae_lambda=gae_lambda, clip_range=clip_range, ent_coef=ent_coef, vf_coef=vf_coef,
                       max_grad_norm=max_grad_norm, normalize_advantage=normalize_advantage, seed=seed,
                       world_size=self.world, net_arch=list(pk["net_arch"]))
        # per-rank streams: minibatch permutations, and the rollout's action sampling -- every rank starts from the
        # same broadcast weights (and often identical arenas), so a shared seed would make the ranks' rollouts
        # bit-identical and shrink the effective batch by the world size
        rank = self.dist.get_rank() if self.dist else 0
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed + 1000 * rank)
        self.sample_gen = torch.Generator(device=self.device)
        self.sample_gen.manual_seed(seed + 7919 * (rank + 1))
        self.num_timesteps = 0
        self._last_obs = None
        self._last_starts = None
        self.logs = []

    # ------------------------------------------------------------------ rollout
    @torch.no_grad()
    def collect_rollouts(self):
        env, pol, T, N = self.env, self.policy, self.hp["n_steps"], self.env.num_envs
        dev = self.device
        if self._last_obs is None:
            env.reset()
            self._last_obs = env.obs.clone()
            self._last_starts = torch.ones(N, device=dev)
        A = pol.action_dim
        buf = dict(obs=torch.empty(T, N, env.obs_dim, device=dev), actions=torch.empty(T, N, A, device=dev),
                   rewards=torch.empty(T, N, device=dev), starts=torch.empty(T, N, device=dev),
                   values=torch.empty(T, N, device=dev), logp=torch.empty(T, N, device=dev))
        ep_r = torch.zeros((), dtype=torch.float64, device=dev)
        ep_n = torch.zeros((), dtype=torch.float64, device=dev)
        for t in range(T):
            obs = self._last_obs
            actions, values, logp = pol(obs, generator=self.sample_gen)
            step_a = actions if pol.discrete else actions.clamp(-1.0, 1.0)
            new_obs, rew, term, trunc = env.step_tensors(step_a.contiguous())
            done = (term | trunc).to(torch.float32)
            buf["obs"][t] = obs
            buf["actions"][t] = actions
            buf["rewards"][t] = rew
            buf["starts"][t] = self._last_starts
            buf["values"][t] = values
            buf["logp"][t] = logp
            # Monitor episodes (r, l) of the arenas that ended this step
            ep_r += (env.ep_return * done).sum()
            ep_n += done.sum().to(torch.float64)
            self._last_obs = new_obs.clone()
            self._last_starts = done
        last_values = pol.predict_values(self._last_obs)
        self.num_timesteps += T * N * self.world
        # GAE(lambda) (RolloutBuffer.compute_returns_and_advantage); truncation never happens in this env
        buf["advantages"], buf["returns"] = compute_gae(buf["rewards"], buf["values"], buf["starts"], last_values,
                                                        self._last_starts, self.hp["gamma"], self.hp["gae_lambda"])
        stats = torch.stack([ep_r, ep_n, buf["rewards"].sum().to(torch.float64)])
        if self.dist:
            self.dist.all_reduce(stats)
        return buf, stats

    # ------------------------------------------------------------------ update
    def train(self, buf):
        hp, pol = self.hp, self.policy
        T, N = buf["rewards"].shape
        n = T * N
        flat = {k: v.reshape(n, *v.shape[2:]) for k, v in buf.items()}
        bs = min(hp["batch_size"], n)
        params = [p for p in pol.parameters()]
        clip = hp["clip_range"]
        last = {}
        for epoch in range(hp["n_epochs"]):
            perm = torch.randperm(n, device=self.device, generator=self.gen)
            for s in range(0, n, bs):
                idx = perm[s:s + bs]
                obs, act = flat["obs"][idx], flat["actions"][idx]
                adv = flat["advantages"][idx]
                norm = hp["normalize_advantage"] and len(adv) > 1
                if norm:  # the global minibatch's mean / unbiased std (torch.std), reduced behind the forward pass
                    st = torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(len(adv)), device=adv.device)])
                    work = self.dist.all_reduce(st, async_op=True) if self.dist else None
                values, logp, ent = pol.evaluate_actions(obs, act)
                if norm:
                    if work is not None:
                        work.wait()
                    m = st[0] / st[2]
                    var = (st[1] - st[2] * m * m) / (st[2] - 1)
                    adv = (adv - m) / (var.clamp_min(0).sqrt() + 1e-8)
                ratio = torch.exp(logp - flat["logp"][idx])
                pl = -torch.min(adv * ratio, adv * ratio.clamp(1 - clip, 1 + clip)).mean()
                vl = torch.nn.functional.mse_loss(flat["returns"][idx], values)
                el = -ent.mean()
                loss = pl + hp["ent_coef"] * el + hp["vf_coef"] * vl
                self.optimizer.zero_grad(set_to_none=False)
                loss.backward()
                if self.dist:  # one fused all-reduce of every gradient, then the mean
                    grads = [p.grad for p in params]
                    flat_allreduce(grads, self.dist)
                    for gr in grads:
                        gr.div_(self.world)
                torch.nn.utils.clip_grad_norm_(params, hp["max_grad_norm"])
                self.optimizer.step()
                last = dict(policy_loss=pl.detach(), value_loss=vl.detach(), entropy_loss=el.detach(),
                            clip_fraction=((ratio - 1).abs() > clip).float().mean().detach())
        return {k: float(v) for k, v in last.items()}

    def learn(self, total_timesteps, log_every=1, callback=None):
        it = 0
        while self.num_timesteps < total_timesteps:
            t0 = time.time()
            buf, stats = self.collect_rollouts()
            t1 = time.time()
            losses = self.train(buf)
            torch.cuda.synchronize(self.device) if self.device.type == "cuda" else None
            t2 = time.time()
            it += 1
            ep_r, ep_n, rsum = (float(x) for x in stats)
            rec = dict(iteration=it, timesteps=self.num_timesteps, ep_rew_mean=ep_r / ep_n if ep_n else None,
                       episodes=int(ep_n), reward_per_step=rsum / (self.hp["n_steps"] * self.env.num_envs * self.world),
                       rollout_s=t1 - t0, train_s=t2 - t1, **losses)
            self.logs.append(rec)
            if callback is not None and callback(self, rec) is False:
                break
        return self

    # ------------------------------------------------------------------ checkpoints (SB3 zip layout, no pickles)
    def save(self, path):
        """zip with policy.pth (a plain state_dict, loadable with weights_only=True) and data (JSON)"""
        with zipfile.ZipFile(path, "w") as z:
            b = io.BytesIO()
            torch.save({k: v.detach().cpu() for k, v in self.policy.state_dict().items()}, b)
            z.writestr("policy.pth", b.getvalue())
            z.writestr("data", json.dumps(dict(self.hp, num_timesteps=self.num_timesteps,
                                               obs_dim=self.policy.obs_dim, action_dim=self.policy.action_dim,
                                               nvec=self.policy.nvec)))

    def load_policy(self, path_or_state):
        sd = load_sb3_policy_state(path_or_state) if isinstance(path_or_state, str) else path_or_state
        self.policy.load_state_dict({k: v.to(self.device) for k, v in sd.items()})
        return self


def compute_gae(rewards, values, starts, last_values, last_starts, gamma, lam):
    """GAE(lambda) over [T, N] device tensors (RolloutBuffer.compute_returns_and_advantage): advantages, returns;
    `starts[t]` = 1 where step t begins an episode, `last_starts` for the step after the buffer"""
    T = rewards.shape[0]
    adv = torch.empty_like(rewards)
    gae = torch.zeros_like(rewards[0])
    for t in reversed(range(T)):
        if t == T - 1:
            nnt, nv = 1.0 - last_starts, last_values
        else:
            nnt, nv = 1.0 - starts[t + 1], values[t + 1]
        delta = rewards[t] + gamma * nv * nnt - values[t]
        gae = delta + gamma * lam * nnt * gae
        adv[t] = gae
    return adv, adv + values


def gae_reference(rewards, values, starts, last_values, last_starts, gamma, lam):
    """plain numpy restatement of RolloutBuffer.compute_returns_and_advantage (test helper)"""
    T = len(rewards)
    adv = np.zeros_like(rewards)
    last = 0.0
    for t in reversed(range(T)):
        if t == T - 1:
            nnt, nv = 1.0 - last_starts, last_values
        else:
            nnt, nv = 1.0 - starts[t + 1], values[t + 1]
        delta = rewards[t] + gamma * nv * nnt - values[t]
        last = delta + gamma * lam * nnt * last
        adv[t] = last
    return adv, adv + values
