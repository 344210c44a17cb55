"""PPO with the reference's API (agent/ppo.py:65-293) on a device-resident rollout.

``PPO(env_fn, config, device)`` / ``.train()`` / ``.save()`` / ``.load()`` and
the per-phase methods keep their reference signatures, so train.py drops in.
What changes underneath:

* the N ``env_fn(i)`` envs become ONE ``RacingVectorEnv`` (rx.envs specs) and
  every rollout step is one batched HIP step, written straight into the
  rollout buffers (obs[t+1], rewards[t], dones[t+1]) -- no host round trip
  per step (the reference does 1 D2H + 3 H2D copies per step, agent/ppo.py:
  114-120);
* GAE is one HIP kernel (rx.gae), bit-exact with compute_advantages;
* episode statistics are summed on the device and read once per update;
* with torch.distributed initialised, each rank owns its env shard and the
  update averages gradients with one all-reduce per optimizer step
  (rx.dist), plus a 4-float all-reduce for the global advantage
  normalisation and the synchronised KL early stop.

Semantics kept on purpose: next-step autoreset, the KL early stop that ends
the WHOLE update (agent/ppo.py:178-182), per-minibatch advantage
normalisation with the unbiased std, np.random.shuffle of b_inds, the linear
lr / log_std anneals, and the speed-weight anneal that the reference applies
to its RecordEpisodeStatistics wrappers only (set
config["apply_speed_weight_anneal"] = True to really apply it).
"""
import contextlib
import json
import os
import random
import types

import numpy as np
import torch
import torch.nn as nn
import torch.optim as optim

from . import _lib
from . import dist as rdist
from .agent import Agent
from .gae import compute_gae
from .optim import FlatAdam


class EpisodeSummary:
    """Device-summed episode statistics of one rollout (replaces the list of
    per-episode dicts agent/ppo.py:121-130 builds on the host)."""

    def __init__(self, sum_return, sum_length, count):
        self.sum_return, self.sum_length, self.count = sum_return, sum_length, int(count)

    def __len__(self):
        return self.count

    def __bool__(self):
        return self.count > 0

    @property
    def mean_reward(self):
        return self.sum_return / self.count if self.count else float("nan")

    @property
    def mean_length(self):
        return self.sum_length / self.count if self.count else float("nan")


def build_vector_env(env_fn, num_envs, seed, device, **kw):
    """Call env_fn(i) for every env (train.py factories) and gather the specs
    into one device vector env, reset (agent/ppo.py:70,85-95)."""
    from .vector_env import RacingVectorEnv
    specs = [env_fn(i) for i in range(num_envs)]
    venv = RacingVectorEnv.from_envs(specs, device=device, seed=seed, **kw)
    venv.reset_device()
    return venv


class PPO:
    log_std_schedule = (-0.5, -1.6)  # agent/ppo.py:250-251
    info_path = "data/training_info_single_3.json"

    def __init__(self, env_fn, config, device="cuda"):
        self.config = config
        want = device if torch.cuda.is_available() and config.get("cuda", True) else "cpu"
        self.device = torch.device(want)
        if self.device.type != "cuda":
            raise RuntimeError("rx.ppo.PPO steps its envs on a HIP device; no CPU env path exists "
                               "(torch.cuda.is_available() is False or config['cuda'] is False)")
        self.env_fn = env_fn
        self.envs = self._make_envs(env_fn)
        random.seed(config["seed"])
        np.random.seed(config["seed"])
        torch.manual_seed(config["seed"])
        self.agent = Agent(self.envs.single_observation_space, self.envs.single_action_space).to(self.device)
        self.optimizer = optim.Adam(self.agent.parameters(), lr=config["learning_rate"], eps=1e-5)
        self._seed_sampling()
        # parameters move into one flat buffer here, BEFORE any graph captures their addresses
        self._flat = FlatAdam(self.agent, self.optimizer, config["max_grad_norm"])
        # one forward now: BLAS handle / kernel-module initialisation belongs to
        # construction, not to the first rollout (no RNG is drawn by get_value)
        with torch.no_grad():
            self.agent.get_value(self.envs.buf["obs"].reshape(-1, self.envs.buf["obs"].shape[-1])[:1])
        self._fresh_obs = True

    def _seed_sampling(self):
        """Data parallel: every rank built the SAME initial policy from
        torch.manual_seed(seed) above, but must draw DIFFERENT action noise /
        device shuffles / random opponent actions -- otherwise rank r's envs
        replay rank 0's (the seed-1 pool repeats tracks, and every env starts on
        its track's start line), and an optimizer step sees ~1/W unique samples.
        The device generator is reseeded with seed + rank (rank 0 keeps the
        single-process stream)."""
        if rdist.world() > 1 and self.device.type == "cuda":
            with torch.cuda.device(self.device):
                torch.cuda.manual_seed(rdist.sampling_seed(self.config["seed"]))

    def _make_envs(self, env_fn):
        c = self.config
        lo, n = rdist.shard(c["num_envs"])
        fn = env_fn if lo == 0 else (lambda i: env_fn(lo + i))
        return build_vector_env(fn, n, c["seed"] + rdist.rank(), self.device)

    @property
    def num_local_envs(self):
        return self.envs.num_envs

    # ------------------------------------------------------------ rollout
    def _policy_ctx(self):
        if self.config.get("policy_dtype", "fp32") == "bf16":
            # no weight-cast cache: the casts must be re-recorded inside captured graphs
            return torch.autocast(device_type="cuda", dtype=torch.bfloat16, cache_enabled=False)
        return contextlib.nullcontext()

    def _fused_rollout(self, T):
        """rx_rollout driver (config["fused_rollout"]: "auto" = up to
        ppo_fused.ROLLOUT_AUTO_MAX_ENVS single-agent envs on the fused fp32
        policy path), else None."""
        from . import ppo_fused
        c = self.config
        if (not c.get("fused_policy", True) or c.get("policy_dtype", "fp32") != "fp32"
                or getattr(self, "_flat", None) is None or not hasattr(self.envs, "_h")
                or not ppo_fused.Rollout.supported(self.envs, self.agent, c)):
            return None
        ro = self.__dict__.get("_rollout")
        if ro is None or ro.T != T or ro.n != self.envs.num_envs:
            ro = self._rollout = ppo_fused.Rollout(self.agent, self._flat, self.envs, T)
        return ro

    def _fused_policy(self, obs):
        """rx_policy_act driver when config["fused_policy"] (default on) and the
        policy is the reference layout in flat fp32 buffers; else None.  With
        config["policy_dtype"] = "bf16" the kernel runs its products on the bf16
        matrix cores (f32 accumulation)."""
        from . import ppo_fused
        c = self.config
        if (not c.get("fused_policy", True) or getattr(self, "_flat", None) is None or obs.dim() != 3
                or not ppo_fused.policy_supported(self.agent, obs.shape[2])):
            return None
        prec = ppo_fused.precision(c)
        pa = self.__dict__.get("_policy_act")
        if pa is None or pa.n != obs.shape[1] or pa.obs_dim != obs.shape[2] or pa.prec != prec:
            pa = self._policy_act = ppo_fused.PolicyAct(self.agent, self._flat, obs.shape[1], obs.shape[2], prec)
        return pa

    def _next_value(self, next_obs):
        """agent.get_value(next_obs).flatten() -- GAE's bootstrap value
        (agent/ppo.py:224-226) -- on the fused policy path from the same
        rx_policy_act kernel that computed the rollout's values (one launch
        instead of the critic's torch GEMMs and activations), with a zero noise
        block (no RNG draw) and scratch action / log-prob rows; torch's forward
        otherwise or with config["fused_next_value"] = False.  With
        config["policy_dtype"] = "bf16" the bootstrap value is the bf16 critic's,
        like every rollout value GAE combines it with (values[t] came from the
        same bf16 kernel), so A_T's delta mixes values of ONE precision; the fp32
        torch critic the reference uses (agent/ppo.py:224) differs from it by the
        bf16 forward's rounding (tests/test_bf16_gpu.py's 2e-2 bound), and
        fused_next_value = False restores it."""
        fp = self._fused_policy(next_obs.unsqueeze(0)) if self.config.get("fused_next_value", True) else None
        if fp is None:
            return self.agent.get_value(next_obs).flatten()
        n = next_obs.shape[0]
        buf = self.__dict__.get("_nv_buf")
        if buf is None or buf[0].shape[0] != n or buf[0].device != next_obs.device:
            z = lambda *s: torch.zeros(s, dtype=torch.float32, device=next_obs.device)  # noqa: E731
            buf = self._nv_buf = (z(n, 2), z(n, 2), z(n))  # noise (zeros), action sink, values
        eps, act, val = buf
        fp(next_obs, act, None, val, eps=eps)
        return val

    def _step_rollout(self, obs):
        """rx_rollout_steps driver (config["rollout_steps"], default "auto" = on)
        for a single-agent handle on the fused policy path, else None."""
        from . import ppo_fused
        c = self.config
        if (self._fused_policy(obs) is None or not ppo_fused.StepRollout.supported(self.envs, self.agent, c)):
            return None
        T, prec = obs.shape[0], ppo_fused.precision(c)
        sr = self.__dict__.get("_steps_rollout")
        if sr is None or sr.T != T or sr.n != self.envs.num_envs or sr.prec != prec:
            sr = self._steps_rollout = ppo_fused.StepRollout(self.agent, self._flat, self.envs, T, prec)
        return sr

    def _rollout_body(self, obs, actions, logprobs, dones, rewards, values, next_obs, next_done):
        T = obs.shape[0]
        obs[0].copy_(next_obs)
        dones[0].copy_(next_done)
        ro = self._fused_rollout(T)
        if ro is not None:  # few envs: the whole rollout is one persistent launch
            ro(obs, actions, logprobs, dones, rewards, values, next_obs, next_done)
            return
        sr = self._step_rollout(obs)
        if sr is not None:  # T x (rx_policy_act + rx_step) enqueued by one library call
            sr(obs, actions, logprobs, dones, rewards, values, next_obs, next_done)
            return
        fused = self._fused_policy(obs)
        for step in range(T):
            if fused is not None:  # one launch: forward, sample, log-prob, value into the buffers
                action = fused(obs[step], actions[step], logprobs[step], values[step])
            else:
                with self._policy_ctx():
                    action, logprob, _, value = self.agent.get_action_and_value(obs[step])
                actions[step].copy_(action)
                logprobs[step].copy_(logprob)
                values[step].copy_(value.flatten())
            last = step + 1 == T
            self.envs.step_device(action,
                                  obs_out=next_obs if last else obs[step + 1],
                                  reward_out=rewards[step],
                                  done_out=next_done if last else dones[step + 1])

    def collect_rollout(self, obs, actions, logprobs, dones, rewards, values, next_obs, next_done):
        """agent/ppo.py:97-132 on the device.  Buffers are [T, N_local, ...].

        With config["graph_rollout"] = True the whole T-step rollout -- noise,
        policy, env kernels -- is captured once into a HIP graph and replayed
        every update (default "auto" = eager: the launches of one step cost
        less host time than their kernels' GPU time, measured down to 16 envs,
        so a capture would only add its one-time cost)."""
        venv = getattr(self.envs, "venv", self.envs)
        T, n = obs.shape[0], obs.shape[1]
        # numpy start draws (two-car envs, config["start_draws"] = "numpy"): one
        # session for the whole rollout, at most one reset per env every other step
        with torch.no_grad(), venv.start_draw_session(T * n // 2 + n):
            # eager by default: with the cached per-step ctypes structs the host
            # keeps ahead of the GPU even at 16 envs, and a capture costs ~0.2 s
            if self._want_graph("graph_rollout", False):
                key = tuple(t.data_ptr() for t in (obs, actions, logprobs, dones, rewards, values, next_obs,
                                                    next_done))
                g = self._graphs.get(key) if hasattr(self, "_graphs") else None
                if g is None:
                    g = self._capture_rollout(key, obs, actions, logprobs, dones, rewards, values, next_obs,
                                              next_done)
                g.replay()
                # the replayed env kernels moved the engine's working state: the
                # env-order arrays must be exported before the next read
                self.envs._launched()
            else:
                self._rollout_body(obs, actions, logprobs, dones, rewards, values, next_obs, next_done)
        s = self.envs.episode_stats(reset=True)
        s = rdist.sum_stats(s, self.device)
        return obs, actions, logprobs, dones, rewards, values, next_obs, next_done, EpisodeSummary(*s)

    def _capture_rollout(self, key, *bufs):
        if not hasattr(self, "_graphs"):
            self._graphs = {}
        obs = bufs[0]
        # warm the policy (BLAS handles, autocast caches) on a side stream without touching the envs
        rng = torch.cuda.get_rng_state(self.device)
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):
                with self._policy_ctx():
                    self.agent.get_action_and_value(obs[0].clone())
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        torch.cuda.set_rng_state(rng, self.device)  # the warm-up must not shift the sampling stream
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):  # records only: no env step executes during capture
            self._rollout_body(*bufs)
        self._graphs[key] = g
        return g

    def compute_advantages(self, rewards, dones, values, next_value, next_done):
        """agent/ppo.py:134-154 as one HIP kernel (bit-exact)."""
        c = self.config
        # persistent outputs: the captured update graph keeps their addresses
        out = self.__dict__.get("_gae_out")
        if out is None or out[0].shape != rewards.shape or out[0].device != rewards.device:
            out = self._gae_out = (torch.empty_like(rewards), torch.empty_like(rewards))
        return compute_gae(rewards, dones, values, next_value, next_done, c["gamma"], c["gae_lambda"], out=out)

    # ------------------------------------------------------------ update
    def _flat_batch(self, advantages, returns, values, logprobs, actions, obs):
        return (obs.reshape((-1,) + obs.shape[2:]), actions.reshape((-1,) + actions.shape[2:]), logprobs.reshape(-1),
                advantages.reshape(-1), returns.reshape(-1), values.reshape(-1))

    def _minibatch_loss(self, b, mb_inds):
        """agent/ppo.py:170-203 for one minibatch -> (loss, approx_kl)."""
        c = self.config
        b_obs, b_actions, b_logprobs, b_advantages, b_returns, b_values = b
        world = rdist.world()
        with self._policy_ctx():
            _, newlogprob, entropy, newvalue = self.agent.get_action_and_value(b_obs[mb_inds], b_actions[mb_inds])
        ratio = (newlogprob - b_logprobs[mb_inds]).exp()
        mb_adv = b_advantages[mb_inds]
        with torch.no_grad():
            if world > 1:  # one 4-float all-reduce: global KL and advantage moments
                stats = rdist.minibatch_stats((b_logprobs[mb_inds] - newlogprob).sum(), mb_adv)
                count = stats[3]
                approx_kl = stats[0] / count
            else:
                approx_kl = (b_logprobs[mb_inds] - newlogprob).mean()
        if world > 1:
            mean = stats[1] / count
            var = (stats[2] - count * mean * mean) / (count - 1)
            mb_adv = (mb_adv - mean) / (var.clamp_min(0).sqrt() + 1e-8)
        else:
            mb_adv = (mb_adv - mb_adv.mean()) / (mb_adv.std() + 1e-8)
        pg_loss = torch.max(-mb_adv * ratio, -mb_adv * torch.clamp(ratio, 1 - c["clip_coef"], 1 + c["clip_coef"])).mean()
        newvalue = newvalue.flatten()
        v_clip = b_values[mb_inds] + torch.clamp(newvalue - b_values[mb_inds], -c["clip_coef"], c["clip_coef"])
        v_loss = 0.5 * torch.max((newvalue - b_returns[mb_inds]) ** 2, (v_clip - b_returns[mb_inds]) ** 2).mean()
        loss = pg_loss + c["ent_coef"] * (-entropy.mean()) + c["vf_coef"] * v_loss
        return loss, approx_kl

    def _early_stop_msg(self, epoch, kl):
        if rdist.rank() == 0:
            print(f"  Early stopping at epoch {epoch + 1} due to KL divergence: {kl:.4f}")

    def _minibatch_size(self):
        world = rdist.world()
        mb = self.config["minibatch_size"]
        return mb // world if world > 1 else mb

    def ppo_update(self, advantages, returns, values, logprobs, actions, obs):
        """agent/ppo.py:156-209; distributed-aware (rx.dist).

        Optimizer step = rx_adam_clip_step (clip_grad_norm_ + Adam in one HIP
        launch on flat buffers, rx.optim).  On one GPU a minibatch step is the
        fused gradient kernel (config["fused_update"], default on) and, with
        config["graph_update"] (default "auto": below 8,192-row minibatches),
        each epoch's minibatch steps are ONE captured HIP graph.  The KL early
        stop is a device flag that turns the remaining optimizer launches into
        no-ops, read by the host once per epoch, so parameters, Adam state and
        np.random consumption end exactly where the reference's immediate
        return leaves them."""
        b = self._flat_batch(advantages, returns, values, logprobs, actions, obs)
        flat = getattr(self, "_flat", None)
        if flat is None:
            return self._update_torch(b)
        flat.rebind()
        flat.sync_lr()
        from . import ppo_fused
        mb = self._minibatch_size()
        fused = self.config.get("fused_update", True) and ppo_fused.supported(self.agent, b, mb)
        if rdist.world() == 1:
            # capture when launches would outpace the GPU work (small minibatches)
            capture = self._want_graph("graph_update", mb < 8192)
            if fused or capture:
                return self._update_epochs(b, fused, capture)
        elif fused:  # data parallel: shard gradients + ONE bucket all-reduce per step, eager
            return self._update_epochs(b, True, False)
        return self._update_flat_eager(b)

    def _want_graph(self, key, auto):
        v = self.config.get(key, "auto")
        return auto if v == "auto" else bool(v)

    def _update_torch(self, b):
        """Reference control flow with torch.optim (no flat buffers: CPU tests)."""
        c = self.config
        B, mb = b[0].shape[0], self._minibatch_size()
        b_inds = np.arange(B)
        params = [p for p in self.agent.parameters()]
        for epoch in range(c["update_epochs"]):
            np.random.shuffle(b_inds)
            perm = torch.from_numpy(b_inds).to(self.device)
            for start in range(0, B, mb):
                loss, approx_kl = self._minibatch_loss(b, perm[start:start + mb])
                if approx_kl > c["kl_target"]:
                    self._early_stop_msg(epoch, float(approx_kl))
                    return
                self.optimizer.zero_grad()
                loss.backward()
                rdist.average_gradients(params)
                nn.utils.clip_grad_norm_(params, c["max_grad_norm"])
                self.optimizer.step()

    def _update_flat_eager(self, b):
        """Eager minibatch loop on the flat optimizer (data parallel: ONE flat
        gradient all-reduce per step; the KL check syncs per minibatch)."""
        c = self.config
        B, mb = b[0].shape[0], self._minibatch_size()
        b_inds = np.arange(B)
        for epoch in range(c["update_epochs"]):
            np.random.shuffle(b_inds)
            perm = torch.from_numpy(b_inds).to(self.device)
            for start in range(0, B, mb):
                loss, approx_kl = self._minibatch_loss(b, perm[start:start + mb])
                if approx_kl > c["kl_target"]:
                    self._early_stop_msg(epoch, float(approx_kl))
                    return
                self._flat.zero_grad()
                loss.backward()
                rdist.average_flat(self._flat.flat_grad)
                self._flat.step()

    def _graph_minibatch(self, b, mb_inds):
        loss, approx_kl = self._minibatch_loss(b, mb_inds)
        hit = (approx_kl > self.config["kl_target"]).reshape(1)
        self._kl_at_stop.copy_(torch.where(hit & ~self._stop, approx_kl.reshape(1).float(), self._kl_at_stop))
        self._stop.logical_or_(hit)
        self._flat.zero_grad()
        loss.backward()
        self._flat.step(stop=self._stop)

    def _epoch_runner(self, b, B, mb, fused, capture):
        """The work of one epoch over the static index tensor ``perm``: with
        ``fused`` (config["fused_update"], default on, reference policy layout)
        a minibatch step is rx_ppo_minibatch_grad + rx_adam_clip_step
        (rx.ppo_fused: 3 launches), otherwise torch autograd + the flat Adam
        launch; with ``capture`` the epoch is one HIP graph.  Cached per
        (buffers, batch, minibatch, dtype, kernel, capture)."""
        from . import ppo_fused
        key = tuple(t.data_ptr() for t in b) + (B, mb, self.config.get("policy_dtype", "fp32"), fused, capture,
                                                self.config.get("shard_update", False))
        graphs = self.__dict__.setdefault("_upd_graphs", {})
        if key in graphs:
            return graphs[key]
        dev = self.device
        ent = types.SimpleNamespace(
            perm=torch.arange(B, device=dev), perm_host=torch.empty(B, dtype=torch.int64).pin_memory(),
            stop=torch.ones(1, dtype=torch.bool, device=dev),  # a warm-up must not move anything
            kl=torch.zeros(1, dtype=torch.float32, device=dev), graph=None, fused=None, run=None)
        if fused:
            ent.fused = ppo_fused.FusedMinibatchGrad(self.agent, self._flat, b, mb, ent.perm, self.config)
            if rdist.world() > 1 or self.config.get("shard_update", False):
                # the data-parallel epoch ("shard_update" runs it on one rank: tests, the bench's
                # world-1 RCCL leg): adv moments -> all-reduce -> finalize, then per optimizer step
                # shard gradient -> bucket all-reduce -> KL check -> Adam.  config["graph_dp"]
                # (default: auto = whenever the process group's collectives are capturable, RCCL)
                # records the whole epoch, collectives included, as ONE HIP graph -- on every
                # rank or on none (rdist.capture_all_or_none): the capture must succeed on all
                # ranks, and its first replay must equal the eager epoch bit for bit on all
                # ranks (parameters, Adam moments, step count, stop flag, KL), else every rank
                # runs the eager launches.  The decision is recorded in rdist.GRAPH_DP.
                w = rdist.world()
                eager = lambda: ent.fused.shard_epoch(ent.stop, ent.kl, w, rdist.all_reduce_sum)  # noqa: E731
                ent.run = eager
                want = self.config.get("graph_dp", "auto")
                if want is True or (want == "auto" and rdist.capturable()):
                    fl = self._flat
                    state = [fl.flat_param, fl.exp_avg, fl.exp_avg_sq, fl.step_t, ent.stop, ent.kl]

                    def capture():
                        eager()  # warm-up with the stop flag up: workspaces, communicator; nothing moves
                        torch.cuda.synchronize(dev)
                        g = torch.cuda.CUDAGraph()
                        try:
                            # thread_local: the process group's watchdog thread may query its
                            # events meanwhile (global mode would invalidate the capture)
                            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                                eager()
                        finally:
                            torch.cuda.synchronize(dev)
                        return g

                    def validate(g):
                        keep = [t.clone() for t in state]

                        def run(fn):
                            ent.stop.zero_()
                            ent.kl.zero_()
                            fn()
                            torch.cuda.synchronize(dev)
                            out = [t.clone() for t in state]
                            for t, k in zip(state, keep):
                                t.copy_(k)
                            return out
                        try:
                            return all(torch.equal(a, b) for a, b in zip(run(eager), run(g.replay)))
                        finally:
                            torch.cuda.synchronize(dev)

                    ent.graph, _ = rdist.capture_all_or_none(capture, validate, device=dev)
                    ent.run = ent.graph.replay if ent.graph is not None else eager
            elif capture:
                ent.graph = torch.cuda.CUDAGraph()
                torch.cuda.synchronize(dev)
                with torch.cuda.graph(ent.graph, capture_error_mode="thread_local"):
                    ent.fused.epoch(ent.stop, ent.kl)
                ent.run = ent.graph.replay
            else:
                ent.run = lambda: ent.fused.epoch(ent.stop, ent.kl)
        else:
            ent.graph = torch.cuda.CUDAGraph()
            self._stop, self._kl_at_stop = ent.stop, ent.kl
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    self._graph_minibatch(b, ent.perm[:mb])
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            with torch.cuda.graph(ent.graph, capture_error_mode="thread_local"):
                for start in range(0, B, mb):
                    self._graph_minibatch(b, ent.perm[start:start + mb])
            ent.run = ent.graph.replay
        graphs[key] = ent
        return ent

    def _device_permutation(self, out):
        """config["shuffle"] = "device": a pseudo-random permutation of the batch
        rows written straight into ``out`` (int64 [B]) by rx_random_permutation
        (Feistel network, include/rx.h), keyed by a draw from torch's CPU
        generator (seeded from config["seed"]) mixed with the rank, so runs
        repeat and data-parallel ranks shuffle independently."""
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) ^ (rdist.rank() * 0x9E3779B97F4A7C15 % 2 ** 64)
        L = _lib.load()
        _lib.check(L.rx_random_permutation(out.numel(), seed, _lib.ptr(out), _lib.stream_ptr(None)),
                   "rx_random_permutation")

    def _update_epochs_async(self, ent, n_mb):
        """Device shuffles on one rank: every epoch (permutation launch + epoch
        graph) is enqueued without waiting for the previous one's KL verdict.
        Once the device stop flag is up, every later launch of the update exits
        at its flag test (k_ppo_grad / k_ppo_reduce / k_adam_apply), so the parameters, the Adam state and
        the step count end exactly as with a host check after every epoch
        (agent/ppo.py:178-182 breaks out of the epoch loop).  The stop epoch
        comes from the optimizer steps taken (a stop in epoch e, minibatch m
        leaves e * n_mb + m of them), and torch's CPU generator is rewound to
        just after that epoch's seed draw, so the generator consumes exactly
        what the per-epoch check would have (config["epoch_sync"] = True keeps
        that synchronous loop).  One host sync per update instead of one per
        epoch."""
        E = self.config["update_epochs"]
        steps0 = self._flat.step_t.clone()
        rng = []
        f = ent.fused
        B = ent.perm.numel()
        if ent.__dict__.get("perms") is None:
            ent.perms = torch.empty((E, B), dtype=torch.int64, device=ent.perm.device)
            ent.stats_all = torch.empty((E, f.n_mb, 2), dtype=torch.float32, device=ent.perm.device)
        # every epoch's permutation up front (the same draws, in the same order),
        # then the advantage statistics of all epochs in ONE launch
        for e in range(E):
            rng.append(torch.get_rng_state())
            self._device_permutation(ent.perms[e])
        f.epochs_stats(ent.perms, ent.stats_all)
        self._epochs_all(ent, E)()
        if bool(ent.stop.item()):
            taken = int(round(float((self._flat.step_t - steps0).item())))
            epoch = min(taken // n_mb, E - 1)
            if epoch + 1 < E:
                torch.set_rng_state(rng[epoch + 1])
            self._early_stop_msg(epoch, float(ent.kl.item()))

    def _epochs_all(self, ent, E):
        """All E epochs' minibatch steps, epoch e reading its rows of ent.perms /
        ent.stats_all in place (FusedMinibatchGrad.epoch_view: no per-epoch copy
        into the runner's buffers) -- ONE HIP graph for the whole update when the
        epoch runner captures graphs (round 6: was a 4 MB perm copy, a stats copy
        and a graph replay per epoch)."""
        run = ent.__dict__.get("run_all")
        if run is None:
            f = ent.fused
            views = [f.epoch_view(ent.perms[e], ent.stats_all[e]) for e in range(E)]

            def steps():
                for e in range(E):
                    for m in range(f.n_mb):
                        f.update(m, ent.stop, ent.kl, batch=views[e])
            if ent.graph is not None:
                g = torch.cuda.CUDAGraph()
                torch.cuda.synchronize(ent.perm.device)
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    steps()
                run = g.replay
                ent.graph_all = g
            else:
                run = steps
            ent.views = views
            ent.run_all = run
        return run

    def _update_epochs(self, b, fused, capture):
        c = self.config
        B, mb = b[0].shape[0], self._minibatch_size()
        ent = self._epoch_runner(b, B, mb, fused, capture)
        device_shuffle = c.get("shuffle", "numpy") == "device"
        b_inds = np.arange(B)
        nxt = None
        ent.stop.zero_()
        if (device_shuffle and ent.fused is not None and rdist.world() == 1 and not c.get("epoch_sync", False)
                and not c.get("shard_update", False)):
            self._update_epochs_async(ent, B // mb)
            return
        for epoch in range(c["update_epochs"]):
            if device_shuffle:  # rx_random_permutation: one launch, no host shuffle / H2D copy
                self._device_permutation(ent.perm)
            else:
                if nxt is None:
                    np.random.shuffle(b_inds)
                else:
                    b_inds = nxt
                ent.perm_host.numpy()[:] = b_inds
                ent.perm.copy_(ent.perm_host, non_blocking=True)
            ent.run()
            rng = None
            if not device_shuffle and epoch + 1 < c["update_epochs"]:
                # shuffle the next epoch while this one runs; undone if it stopped
                rng = np.random.get_state()
                nxt = b_inds.copy()
                np.random.shuffle(nxt)
            if bool(ent.stop.item()):
                if rng is not None:
                    np.random.set_state(rng)
                self._early_stop_msg(epoch, float(ent.kl.item()))
                return

    # ------------------------------------------------------------ driver
    def _anneal(self, update, num_updates):
        c = self.config
        frac = max(0.0, 1.0 - update / num_updates)
        self.optimizer.param_groups[0]["lr"] = frac * c["learning_rate"]
        lo, hi = self.log_std_schedule
        self.agent.log_std.data.fill_(frac * lo + (1 - frac) * hi)
        return frac

    def _speed_weight_anneal(self, frac):
        w = 8.0 + (1 - frac) * 6.0  # agent/ppo.py:256
        if self.config.get("apply_speed_weight_anneal", False):
            self.envs.set_speed_weight(w)
        return w

    def _buffers(self):
        c = self.config
        T, N = c["num_steps"], self.num_local_envs
        obs_shape = tuple(self.envs.single_observation_space.shape)
        act_shape = tuple(self.envs.single_action_space.shape)
        z = lambda *s: torch.zeros(s, device=self.device)  # noqa: E731
        return (z(T, N, *obs_shape), z(T, N, *act_shape), z(T, N), z(T, N), z(T, N), z(T, N))

    def train_iter(self):
        """agent/ppo.py:211-281 as a generator: yields (update, num_updates,
        global_step, EpisodeSummary) after every update (evaluation hooks)."""
        c = self.config
        obs, actions, logprobs, dones, rewards, values = self._buffers()
        next_obs = self.envs.buf["obs"].clone()  # obs of the reset done at construction
        next_done = torch.zeros(self.num_local_envs, device=self.device)
        num_updates = c["total_timesteps"] // c["batch_size"]
        global_step = 0
        for update in range(num_updates):
            frac = self._anneal(update, num_updates)
            self._speed_weight_anneal(frac)
            obs, actions, logprobs, dones, rewards, values, next_obs, next_done, ep = self.collect_rollout(
                obs, actions, logprobs, dones, rewards, values, next_obs, next_done)
            with torch.no_grad():
                next_value = self._next_value(next_obs)
            advantages, returns = self.compute_advantages(rewards, dones, values, next_value, next_done)
            self.ppo_update(advantages, returns, values, logprobs, actions, obs)
            global_step += c["batch_size"]
            yield update, num_updates, global_step, ep

    def train(self):
        training_info = {"steps": [], "rewards": []}
        for update, num_updates, global_step, ep in self.train_iter():
            self._log(update, num_updates, global_step, ep, training_info)
        self._save_info(training_info)
        return training_info

    def _log(self, update, num_updates, global_step, ep, info, extra=""):
        if ep:
            info["steps"].append(global_step)
            info["rewards"].append(float(ep.mean_reward))
            if rdist.rank() == 0:
                print(f"Update {update + 1}/{num_updates} | Step {global_step} | Episodes: {len(ep)} | "
                      f"Mean Reward: {ep.mean_reward:.2f} | Mean Length: {ep.mean_length:.2f}{extra}")
        elif rdist.rank() == 0:
            print(f"Update {update + 1}/{num_updates} | Step {global_step} | No episodes completed this rollout")

    def _save_info(self, info):
        if rdist.rank() != 0:
            return
        try:
            with open(self.info_path, "w") as f:
                json.dump(info, f)
            print(f"\nTraining data saved to {self.info_path}")
        except Exception as e:  # noqa: BLE001 -- agent/ppo.py:282-287 behaviour
            print(f"Warning: Could not save data: {e}")

    def save(self, path):
        d = os.path.dirname(path)
        if d and not os.path.isdir(d):
            os.makedirs(d, exist_ok=True)
        torch.save(self.agent.state_dict(), path)

    def load(self, path):
        self.agent.load_state_dict(torch.load(path, map_location=self.device, weights_only=True))
