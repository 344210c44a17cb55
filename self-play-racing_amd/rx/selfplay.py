"""Two-car self-play (BASELINE.json configs[3]) -- environment/wrappers.py:5-63
and agent/self_play_ppo.py:8-187 on the device.

``SelfPlayVectorEnv`` exposes agent 0 of N two-car envs as N single-agent
envs, like N ``SelfPlayWrapper``s inside a SyncVectorEnv, but the opponent
(agent 1) is driven by ONE batched forward of the frozen policy over all N
envs per step (the reference runs a batch-1 forward with a host round trip
per env per step, wrappers.py:36-39), or by uniform random actions drawn on
the device when the pool is empty (wrappers.py:32-33; Box([-1, 0], [1, 1]),
so throttle in [0, 1] maps to (a+1)/2 in [0.5, 1] inside the env).

``SelfPlayPPO`` keeps the reference's pool mechanics: snapshot every
``snapshot_freq`` updates into a FIFO pool of ``pool_size``, an opponent drawn
with np.random.choice per update (None while the pool is empty), envs rebuilt
(= reset) every update while next_obs is left stale (SURVEY.md §8 Q10;
config["refresh_obs_on_rebuild"] = True fixes it), a full checkpoint every 10
updates, and ``train(resume_from=...)``.
"""
import copy
import json

import numpy as np
import torch

from . import dist as rdist
from .agent import Agent
from .ppo import PPO, EpisodeSummary


class SelfPlayVectorEnv:
    def __init__(self, venv, agent_idx=0, seed=0):
        if venv.n_agents != 2:
            raise ValueError("self-play needs a 2-car vector env")
        self.venv = venv
        self.agent_idx = agent_idx
        self.opp_idx = 1 - agent_idx
        self.num_envs = venv.num_envs
        self.device = venv.device
        self.single_observation_space = venv.single_observation_space
        self.single_action_space = venv.single_action_space
        self.envs = venv.envs
        self.opponent_policy = None
        self._opp_fused = None
        self._act = torch.zeros((self.num_envs, 2, 2), dtype=torch.float32, device=self.device)
        self.buf = {"obs": self.venv.buf["obs"][:, agent_idx]}

    def set_opponent(self, policy, flat=None, prec=0):
        """policy: an Agent (or None = random actions).  With ``flat`` (an
        rx.optim.FlatParams of that policy) the opponent's forward + sampling is
        one rx_policy_act launch reading the two-car obs buffer in place
        (``prec``: RX_PREC_FP32 / RX_PREC_BF16 matrix-core precision)."""
        from . import ppo_fused
        self.opponent_policy = policy
        self._opp_fused = None
        if policy is not None and flat is not None and ppo_fused.policy_supported(policy, self.venv.D):
            self._opp_fused = ppo_fused.PolicyAct(policy, flat, self.num_envs, self.venv.D, prec)

    def _opponent_actions(self):
        o = self._act[:, self.opp_idx]
        if self.opponent_policy is None:
            u = torch.rand((self.num_envs, 2), device=self.device)  # default generator: graph-capturable
            u[:, 0].mul_(2.0).sub_(1.0)  # steer ~ U(-1, 1); throttle ~ U(0, 1)
            o.copy_(u)
        elif self._opp_fused is not None:  # writes agent 1's actions straight into _act
            self._opp_fused(self.venv.buf["obs"][:, self.opp_idx], o)
        else:
            with torch.no_grad():
                a = self.opponent_policy.get_action_and_value(self.venv.buf["obs"][:, self.opp_idx])[0]
            o.copy_(a)

    def reset_device(self):
        self.venv.reset_device()
        return self.venv.buf["obs"][:, self.agent_idx]

    def step_device(self, actions, obs_out=None, reward_out=None, done_out=None, **kw):
        self._opponent_actions()
        self._act[:, self.agent_idx].copy_(actions)
        obs, rew, done = self.venv.step_device(self._act, done_out=done_out, **kw)
        o = obs[:, self.agent_idx]
        r = rew[:, self.agent_idx]
        if obs_out is not None:
            obs_out.copy_(o)
            o = obs_out
        if reward_out is not None:
            reward_out.copy_(r)
            r = reward_out
        return o, r, done  # done = dones['__all__'] (wrappers.py:51) = terminated | truncated

    def episode_stats(self, reset=True):
        return self.venv.episode_stats(reset)

    def _launched(self, stream=None):
        """A replayed rollout graph moved the two-car handle's working state."""
        self.venv._launched(stream)

    def close(self):
        self.venv.close()


class SelfPlayPPO(PPO):
    log_std_schedule = (-0.3, -1.2)  # agent/self_play_ppo.py:128-129
    info_path = "data/training_info_self_play_3.json"
    checkpoint_fmt = "models/checkpoint_update_{}.pth"

    def __init__(self, env_fn, config, device="cuda"):
        self.opponent_pool = []
        self.curr_opponent = None
        self.snapshot_freq = config["snapshot_freq"]
        self.pool_size = config["pool_size"]
        super().__init__(env_fn, config, device)

    def _make_envs(self, env_fn):
        from .ppo import build_vector_env
        c = self.config
        lo, n = rdist.shard(c["num_envs"])
        fn = env_fn if lo == 0 else (lambda i: env_fn(lo + i))
        venv = build_vector_env(fn, n, c["seed"] + rdist.rank(), self.device)
        if c.get("start_draws", "hash") == "numpy":  # the reference's np.random start-slot stream
            if rdist.world() > 1:
                # every rank would replay the SAME np.random stream for its own env shard, not
                # the reference's single stream over the global env order
                raise ValueError("start_draws='numpy' needs world size 1: the reference's single "
                                 "np.random start-slot stream cannot be split over ranks (use 'hash')")
            venv.use_numpy_start_draws()
        return SelfPlayVectorEnv(venv, 0, seed=c["seed"] + rdist.rank())

    def snapshot_agent(self):
        """A frozen copy of the current policy (agent/self_play_ppo.py:31-44 builds a
        fresh Agent and loads a deep copy of the state dict).  Here: ONE deepcopy of
        the module -- each parameter and buffer is cloned on the device (one
        device-to-device copy each; gradients are not copied) -- instead of a CPU
        orthogonal init, 13 pageable host-to-device copies (each one a stream sync)
        and 13 state-dict copies."""
        snap = copy.deepcopy(self.agent)
        snap.eval()
        for p in snap.parameters():
            p.grad = None
            p.requires_grad = False
        return snap

    def advance_pool(self, update):
        """agent/self_play_ppo.py:115-122: snapshot every snapshot_freq updates
        (not at update 0) into the FIFO pool of pool_size."""
        if update > 0 and update % self.snapshot_freq == 0:
            self.opponent_pool.append(self.snapshot_agent())
            if len(self.opponent_pool) > self.pool_size:
                self.opponent_pool.pop(0)

    @staticmethod
    def checkpoint_due(update):
        """agent/self_play_ppo.py:154: a full checkpoint every 10 updates, not at 0."""
        return update > 0 and update % 10 == 0

    def select_opponent(self):
        if not self.opponent_pool:
            return None
        return self.opponent_pool[np.random.choice(len(self.opponent_pool))]

    def update_opponent(self):
        """agent/self_play_ppo.py:46-50: pick an opponent and rebuild (= reset) the envs.

        The chosen pool member's weights are copied into one static opponent
        module, so a graph-captured rollout keeps valid parameter addresses."""
        self.curr_opponent = self.select_opponent()
        if self.curr_opponent is None:
            self.envs.set_opponent(None)
        else:
            if getattr(self, "_opp_static", None) is None:
                from .optim import FlatParams
                self._opp_static = self.snapshot_agent()
                self._opp_flat = FlatParams(self._opp_static)  # before any graph captures its addresses
            with torch.no_grad():
                for dst, src in zip(self._opp_static.state_dict().values(), self.curr_opponent.state_dict().values()):
                    dst.copy_(src)
            from . import ppo_fused
            fused = self.config.get("fused_policy", True)
            self.envs.set_opponent(self._opp_static, self._opp_flat if fused else None, ppo_fused.precision(self.config))
        self.envs.reset_device()

    def _step_rollout(self, obs):
        """rx_selfplay_rollout_steps driver (config["rollout_steps"], default on)
        while the opponent is a frozen policy on rx_policy_act; the random
        opponent of an empty pool keeps the per-step path."""
        from . import ppo_fused
        c = self.config
        if self._fused_policy(obs) is None or not ppo_fused.SelfPlayStepRollout.supported(self.envs, self.agent, c):
            return None
        T, prec = obs.shape[0], ppo_fused.precision(c)
        sr = self.__dict__.get("_sp_steps_rollout")
        if sr is None or sr.T != T or sr.n != self.envs.num_envs or sr.prec != prec:
            sr = self._sp_steps_rollout = ppo_fused.SelfPlayStepRollout(self.agent, self._flat, self.envs, T, prec)
        return sr

    def collect_rollout(self, *bufs):
        # one captured graph per opponent kind (random vs frozen policy): the kind
        # changes control flow inside the step, the weights do not (static module)
        graphs = getattr(self, "_graphs_by_kind", {})
        kind = self.envs.opponent_policy is not None
        self._graphs = graphs.setdefault(kind, {})
        self._graphs_by_kind = graphs
        return super().collect_rollout(*bufs)

    def load_checkpoint(self, path):
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.agent.load_state_dict(ck["agent_state_dict"])
        self.optimizer.load_state_dict(ck["optimizer_state_dict"])
        self._flat.import_state()
        self.opponent_pool = []
        for sd in ck["opponent_pool"]:
            o = Agent(self.envs.single_observation_space, self.envs.single_action_space).to(self.device)
            o.load_state_dict(sd)
            o.eval()
            for p in o.parameters():
                p.requires_grad = False
            self.opponent_pool.append(o)
        info = ck.get("training_info", {"steps": [], "rewards": [], "opponent_pool_size": []})
        return ck["update"], ck["global_step"], info

    def train_iter(self, resume_from=None):
        """agent/self_play_ppo.py:70-187 as a generator: yields (update,
        num_updates, global_step, EpisodeSummary, info) after every update.
        config["checkpoint"] = False skips the every-10-updates checkpoint files
        (benchmarks); the default keeps the reference's cadence."""
        c = self.config
        obs, actions, logprobs, dones, rewards, values = self._buffers()
        next_obs = self.envs.buf["obs"].clone()
        next_done = torch.zeros(self.num_local_envs, device=self.device)
        num_updates = c["total_timesteps"] // c["batch_size"]
        if resume_from:
            start, global_step, info = self.load_checkpoint(resume_from)
            start += 1
        else:
            start, global_step = 0, 0
            info = {"steps": [], "rewards": [], "opponent_pool_size": []}
        self._iter_info = info
        # phase_ms (benchmarks): a dict to receive the last update's phase times, each
        # phase bracketed by device syncs (None = no syncs, the normal path)
        mark = self._phase_mark
        for update in range(start, num_updates):
            mark(None)
            self.advance_pool(update)
            self.update_opponent()
            if c.get("refresh_obs_on_rebuild", False):
                next_obs.copy_(self.envs.buf["obs"])
                next_done.zero_()
            self._anneal(update, num_updates)
            mark("opponent_draw_and_rebuild_ms")
            obs, actions, logprobs, dones, rewards, values, next_obs, next_done, ep = self.collect_rollout(
                obs, actions, logprobs, dones, rewards, values, next_obs, next_done)
            mark("rollout_ms")
            with torch.no_grad():
                next_value = self._next_value(next_obs)
            advantages, returns = self.compute_advantages(rewards, dones, values, next_value, next_done)
            mark("gae_ms")
            self.ppo_update(advantages, returns, values, logprobs, actions, obs)
            mark("update_ms")
            global_step += c["batch_size"]
            if c.get("checkpoint", True) and self.checkpoint_due(update) and rdist.rank() == 0:
                self.save_checkpoint(update, global_step, info)
            yield update, num_updates, global_step, ep, info

    phase_ms = None

    def _phase_mark(self, name):
        if self.phase_ms is None:
            return
        import time
        torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        if name is not None:
            self.phase_ms[name] = round((now - self._phase_t) * 1e3, 3)
        self._phase_t = now

    def train(self, resume_from=None):
        info = None
        for update, num_updates, global_step, ep, info in self.train_iter(resume_from):
            if ep:
                info["opponent_pool_size"].append(len(self.opponent_pool))
            self._log(update, num_updates, global_step, ep, info, extra=f" | Pool Size: {len(self.opponent_pool)}")
        if info is None:  # resumed past the last update: the checkpoint's info
            info = self._iter_info
        self._save_info(info)
        return info

    def save_checkpoint(self, update, global_step, info, path=None):
        """agent/self_play_ppo.py:146-159 checkpoint dict."""
        import os
        path = path or self.checkpoint_fmt.format(update)
        d = os.path.dirname(path)
        self._flat.export_state()
        try:
            if d:
                os.makedirs(d, exist_ok=True)
            torch.save({"update": update, "global_step": global_step, "agent_state_dict": self.agent.state_dict(),
                        "optimizer_state_dict": self.optimizer.state_dict(),
                        "opponent_pool": [o.state_dict() for o in self.opponent_pool],
                        "config": json.loads(json.dumps(self.config)), "training_info": info}, path)
        except OSError as e:
            print(f"Warning: could not save checkpoint: {e}")
        return path


__all__ = ["SelfPlayVectorEnv", "SelfPlayPPO", "EpisodeSummary"]
