"""Driver of the fused PPO minibatch gradient (include/rx.h rx_ppo_*).

``FusedMinibatchGrad`` binds one flattened rollout (obs, actions, logprobs,
advantages, returns, values -- persistent buffers), the flat policy
parameters of rx.optim.FlatAdam and the epoch's index tensor, and issues per
epoch: one rx_ppo_adv_stats_ws call (every minibatch's advantage mean/std),
then per minibatch rx_ppo_minibatch_update (forward + loss + backward,
split-K reduce + KL check + clip norms, Adam).  Everything is enqueued on
the current stream with no host sync, so PPO captures an epoch as one graph.
"""
import torch

from . import _lib


def precision(config):
    """Matrix-core precision of the fused policy kernels: config["policy_dtype"]
    "fp32" (exact f32 MFMA, default) or "bf16" (bf16 operands, f32 accumulation)."""
    dt = config.get("policy_dtype", "fp32")
    if dt not in _lib.PRECISION:
        raise ValueError(f"policy_dtype={dt!r}: 'fp32' or 'bf16'")
    return _lib.PRECISION[dt]


def supported(agent, b, mb):
    """True when the fused kernel covers this policy / batch: the reference
    Agent layout (64-wide tanh trunks, 2 actions, D in {15, 19}), float32,
    and a batch that splits into whole minibatches."""
    obs = b[0]
    if obs.dim() != 2 or obs.shape[1] not in (15, 19) or b[1].shape[-1] != 2:
        return False
    B = obs.shape[0]
    if mb <= 0 or B % mb or any(t.dtype != torch.float32 or not t.is_contiguous() for t in b):
        return False
    L = _lib.load()
    n = sum(p.numel() for p in agent.parameters())
    return n == L.rx_ppo_n_params(obs.shape[1])


class FusedMinibatchGrad:
    def __init__(self, agent, flat, b, mb, perm, config):
        L = _lib.load()
        self.L = L
        obs, actions, logprobs, advantages, returns, values = b
        B, D = obs.shape
        self.n_mb = B // mb
        self.mb = mb
        dev = obs.device
        self.stats = torch.zeros(2 * self.n_mb, dtype=torch.float32, device=dev)
        self.ws_f = torch.empty(L.rx_ppo_workspace_floats(D, mb), dtype=torch.float32, device=dev)
        self.ws_d = torch.empty(L.rx_ppo_workspace_doubles(mb), dtype=torch.float64, device=dev)
        # partial advantage moments (rx_ppo_adv_stats_ws), sized for every epoch's minibatches at once
        self.adv_ws = torch.empty(L.rx_ppo_adv_workspace_doubles(mb, max(1, int(config["update_epochs"])) * self.n_mb),
                                  dtype=torch.float64, device=dev)
        self.flat = flat
        self._keep = (b, perm, agent.log_std)  # the struct holds raw pointers into these
        self.batch = _lib.RxPPOBatch(D, mb, B, _lib.ptr(obs), _lib.ptr(actions), _lib.ptr(logprobs),
                                     _lib.ptr(advantages), _lib.ptr(returns), _lib.ptr(values), _lib.ptr(perm),
                                     _lib.ptr(flat.flat_param), _lib.ptr(agent.log_std), _lib.ptr(self.stats),
                                     float(config["clip_coef"]), float(config["vf_coef"]), float(config["kl_target"]),
                                     precision(config))

    def adv_stats(self, stream=None):
        """Every minibatch's advantage (mean, unbiased std) for the current perm:
        rx_ppo_adv_stats_ws, chunks of 2,048 rows on their own workgroups."""
        _lib.check(self.L.rx_ppo_adv_stats_ws(self.batch, self.n_mb, _lib.ptr(self.adv_ws), _lib.ptr(self.stats), None,
                                              _lib.stream_ptr(stream)), "rx_ppo_adv_stats_ws")

    def grad(self, m, stop, kl_at_stop, stream=None):
        _lib.check(self.L.rx_ppo_minibatch_grad(self.batch, int(m), _lib.ptr(self.ws_f), _lib.ptr(self.ws_d),
                                                _lib.ptr(self.flat.flat_grad), _lib.ptr(stop), _lib.ptr(kl_at_stop),
                                                _lib.stream_ptr(stream)), "rx_ppo_minibatch_grad")

    def shard_epoch(self, stop, kl_at_stop, world, all_reduce):
        """One epoch of a data-parallel update over this rank's shard: the
        minibatch advantage moments are all-reduced once per epoch, then per
        minibatch the shard gradient and KL (pre-scaled by 1/world) go out in
        ONE all-reduce of FlatAdam.bucket, followed by the KL check and the
        Adam launch.  ``all_reduce`` is an in-place SUM (rx.dist.all_reduce_sum)."""
        L, s = self.L, _lib.stream_ptr(None)
        mom = self.__dict__.get("moments")
        if mom is None:
            mom = self.moments = torch.empty((self.n_mb, 2), dtype=torch.float64, device=self.stats.device)
        _lib.check(L.rx_ppo_adv_stats_ws(self.batch, self.n_mb, _lib.ptr(self.adv_ws), None, _lib.ptr(mom), s),
                   "rx_ppo_adv_stats_ws")
        all_reduce(mom)
        _lib.check(L.rx_ppo_adv_finalize(_lib.ptr(mom), self.n_mb, self.mb * world, _lib.ptr(self.stats), s),
                   "rx_ppo_adv_finalize")
        flat, scale = self.flat, 1.0 / world
        for m in range(self.n_mb):
            _lib.check(L.rx_ppo_minibatch_grad_shard(self.batch, m, scale, _lib.ptr(self.ws_f), _lib.ptr(self.ws_d),
                                                     _lib.ptr(flat.flat_grad), _lib.ptr(flat.kl_slot), _lib.ptr(stop),
                                                     s), "rx_ppo_minibatch_grad_shard")
            all_reduce(flat.bucket)
            _lib.check(L.rx_ppo_kl_check(_lib.ptr(flat.kl_slot), self.batch.kl_target, _lib.ptr(stop),
                                         _lib.ptr(kl_at_stop), s), "rx_ppo_kl_check")
            flat.step(stop=stop)

    def update(self, m, stop, kl_at_stop, stream=None, batch=None):
        """One optimizer step on minibatch m (rx_ppo_minibatch_update: gradient,
        reduce + clip norms + step count, Adam: three launches); ``batch``: a view
        of self.batch with another epoch's perm / stats rows (epoch_view)."""
        f = self.flat
        ws = self.__dict__.get("adam_ws")
        if ws is None:
            n = self.L.rx_ppo_update_workspace_floats(self.batch.obs_dim, f.cfg)
            if n == 0:
                raise RuntimeError(self.L.rx_last_error().decode())
            # zero-filled: its last word is the fused launch's arrival counter (rx.h, ABI v22)
            ws = self.adam_ws = torch.zeros(n, dtype=torch.float32, device=self.stats.device)
        _lib.check(self.L.rx_ppo_minibatch_update(
            self.batch if batch is None else batch, int(m), f.cfg, _lib.ptr(f.flat_param), _lib.ptr(self.ws_f), _lib.ptr(self.ws_d),
            _lib.ptr(f.flat_grad), _lib.ptr(f.exp_avg), _lib.ptr(f.exp_avg_sq), _lib.ptr(f.step_t), _lib.ptr(f.lr_t),
            _lib.ptr(stop), _lib.ptr(kl_at_stop), _lib.ptr(ws), _lib.stream_ptr(stream)), "rx_ppo_minibatch_update")

    def epoch(self, stop, kl_at_stop, stats=True):
        """All minibatch steps of one epoch over the current perm (``stats``:
        its advantage statistics first; False when the caller has already put
        them in ``self.stats``, see epochs_stats)."""
        if stats:
            self.adv_stats()
        for m in range(self.n_mb):
            self.update(m, stop, kl_at_stop)

    def epoch_view(self, perm, stats):
        """self.batch reading its minibatch rows from ``perm`` (int64 [B]) and its
        advantage statistics from ``stats`` (float32 [n_mb, 2]) in place -- one
        epoch's rows of the [E, B] / [E, n_mb, 2] buffers of epochs_stats, with no
        copy into self.batch's own buffers.  The caller keeps both alive."""
        b = RxPPOBatch_copy(self.batch)
        b.perm = _lib.ptr(perm)
        b.adv_stats = _lib.ptr(stats)
        return b

    def epochs_stats(self, perms, stats_out, stream=None):
        """Advantage statistics of E epochs in ONE rx_ppo_adv_stats_ws call:
        ``perms`` int64 [E, B] (one permutation per epoch), ``stats_out``
        float32 [E, n_mb, 2].  Workgroup e * n_mb + m sums minibatch m of epoch
        e exactly as the per-epoch launch does (same rows, same order), so the
        rows equal E separate launches bit for bit; E * n_mb workgroups keep
        that many CUs gathering instead of n_mb.  The batch view addresses the
        E * B indices (every index is still < B: they are permutations)."""
        E, B = perms.shape
        b = RxPPOBatch_copy(self.batch)
        b.perm = _lib.ptr(perms)
        b.n_rows = E * B
        self._keep_epochs = (perms, stats_out)
        need = self.L.rx_ppo_adv_workspace_doubles(self.mb, E * self.n_mb)
        if self.adv_ws.numel() < need:
            # a graph captured over adv_stats() / shard_epoch() holds the old buffer's
            # address: keep it alive for the lifetime of this object, never free it
            self.__dict__.setdefault("_retired_ws", []).append(self.adv_ws)
            self.adv_ws = torch.empty(need, dtype=torch.float64, device=self.adv_ws.device)
        _lib.check(self.L.rx_ppo_adv_stats_ws(b, E * self.n_mb, _lib.ptr(self.adv_ws), _lib.ptr(stats_out), None,
                                              _lib.stream_ptr(stream)), "rx_ppo_adv_stats_ws")


def RxPPOBatch_copy(b):
    c = _lib.RxPPOBatch()
    for name, _ in _lib.RxPPOBatch._fields_:
        setattr(c, name, getattr(b, name))
    return c


class PolicyAct:
    """rx_policy_act driver: one launch per rollout step instead of ~20 torch
    launches.  The N(0, 1) noise is drawn with torch's normal_() into a
    persistent [N, 2] buffer, exactly the draw Normal.sample() makes
    (torch.normal(mu, std) = normal_() * std + mu), so the sampling stream is
    unchanged; mu / value differ from the torch forward by float rounding."""

    def __init__(self, agent, flat, n, obs_dim, prec=_lib.RX_PREC_FP32):
        self.L = _lib.load()
        self.agent, self.flat, self.n, self.obs_dim = agent, flat, int(n), int(obs_dim)
        self.prec = int(prec)
        dev = flat.flat_param.device
        self.eps = torch.empty((self.n, 2), dtype=torch.float32, device=dev)
        self._lp = torch.empty(self.n, dtype=torch.float32, device=dev)  # sinks when the caller
        self._val = torch.empty(self.n, dtype=torch.float32, device=dev)  # wants actions only
        self._io_cache = {}

    @staticmethod
    def _rows(t, n, width, name):
        """Row stride (floats) of a float32 [n, width] view whose rows may be spaced out."""
        if t.dtype != torch.float32 or t.dim() != 2 or tuple(t.shape) != (n, width) or t.stride(1) != 1:
            raise ValueError(f"rx_policy_act: {name} must be a float32 [{n}, {width}] view with unit column "
                             f"stride, got {tuple(t.shape)} / {t.stride()}")
        return t.stride(0)

    def __call__(self, obs, actions_out, logprobs_out=None, values_out=None, stream=None, eps=None):
        """``eps``: a caller-drawn float32 [n, 2] N(0, 1) block (e.g. one slice of
        a rollout's noise drawn up front); default: draw into the own buffer."""
        lp = self._lp if logprobs_out is None else logprobs_out
        val = self._val if values_out is None else values_out
        if eps is not None and (tuple(eps.shape) != (self.n, 2) or eps.dtype != torch.float32
                                or not eps.is_contiguous()):
            raise ValueError("rx_policy_act: eps must be a contiguous float32 [n, 2] block")
        e = self.eps if eps is None else eps
        key = (obs.data_ptr(), actions_out.data_ptr(), lp.data_ptr(), val.data_ptr(), e.data_ptr())
        io = self._io_cache.get(key) if self._io_cache.get("shapes") == (obs.shape, obs.stride(),
                                                                         actions_out.stride()) else None
        if io is None:  # validate once per buffer set (a rollout reuses the same rows every update)
            os_ = self._rows(obs, self.n, self.obs_dim, "obs")
            as_ = self._rows(actions_out, self.n, 2, "actions")
            for t in (lp, val):
                if tuple(t.shape) != (self.n,) or t.dtype != torch.float32 or not t.is_contiguous():
                    raise ValueError("rx_policy_act: log-prob / value outputs must be contiguous float32 [n]")
            if len(self._io_cache) > 8192:
                self._io_cache.clear()
            self._io_cache["shapes"] = (obs.shape, obs.stride(), actions_out.stride())
            io = self._io_cache[key] = _lib.RxPolicyIO(
                self.obs_dim, self.n, _lib.view_ptr(obs), _lib.ptr(e), _lib.ptr(self.flat.flat_param),
                _lib.ptr(self.agent.log_std), _lib.view_ptr(actions_out), _lib.ptr(lp), _lib.ptr(val), os_, as_,
                self.prec)
        if eps is None:
            self.eps.normal_()
        _lib.check(self.L.rx_policy_act(io, _lib.stream_ptr(stream)), "rx_policy_act")
        return actions_out


def policy_supported(agent, obs_dim):
    if obs_dim not in (15, 19):
        return False
    return sum(p.numel() for p in agent.parameters()) == _lib.load().rx_ppo_n_params(obs_dim)


class Rollout:
    """rx_rollout driver: a whole T-step rollout of few single-agent envs as
    ONE persistent launch (include/rx.h; k_rollout) instead of T x (noise
    draw + rx_policy_act + two env kernels).  The N(0, 1) noise of all T steps
    is drawn up front with ONE torch normal_() on a [T, N, 2] buffer: the same
    distribution as the per-step draws but a different sample of torch's
    stream; given the same noise, every output equals the per-step fused path
    (rx_policy_act + rx_step) bit for bit (tests/test_rollout_gpu.py)."""

    def __init__(self, agent, flat, venv, T):
        self.L = _lib.load()
        self.agent, self.flat, self.venv, self.T = agent, flat, venv, int(T)
        self.n, self.obs_dim = venv.num_envs, venv.D
        self.eps = torch.empty((self.T, self.n, 2), dtype=torch.float32, device=flat.flat_param.device)
        self._cache = {}

    @staticmethod
    def supported(venv, agent, config):
        if venv.n_agents != 1 or not policy_supported(agent, venv.D):
            return False
        mode = config.get("fused_rollout", "auto")
        if mode is False or mode == "off":
            return False
        if not _lib.load().rx_rollout_supported(venv._h):
            return False
        return mode is True or venv.num_envs <= ROLLOUT_AUTO_MAX_ENVS

    def __call__(self, obs, actions, logprobs, dones, rewards, values, next_obs, next_done, eps=None, stream=None):
        """obs[0] / dones[0] hold the rollout's first observation / done flags;
        fills the rest like collect_rollout's step loop.  ``eps`` (tests): a
        [T, N, 2] noise tensor to use instead of a fresh draw."""
        T, n, D = self.T, self.n, self.obs_dim
        shapes = {"obs": (obs, (T, n, D)), "actions": (actions, (T, n, 2)), "logprobs": (logprobs, (T, n)),
                  "values": (values, (T, n)), "rewards": (rewards, (T, n)), "dones": (dones, (T, n)),
                  "next_obs": (next_obs, (n, D)), "next_done": (next_done, (n,))}
        for k, (t, shp) in shapes.items():
            if tuple(t.shape) != shp or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"rx_rollout: {k} must be a contiguous float32 {shp}, got {tuple(t.shape)} {t.dtype}")
        e = self.eps if eps is None else eps
        key = tuple(t.data_ptr() for t in (obs, actions, logprobs, dones, rewards, values, next_obs, next_done, e))
        r = self._cache.get(key)
        if r is None:
            if len(self._cache) > 64:
                self._cache.clear()
            r = self._cache[key] = _lib.RxRolloutIO(
                T, D, _lib.ptr(self.flat.flat_param), _lib.ptr(self.agent.log_std), _lib.ptr(e), _lib.ptr(obs),
                _lib.ptr(actions), _lib.ptr(logprobs), _lib.ptr(values), _lib.ptr(rewards), _lib.ptr(dones),
                _lib.ptr(next_obs), _lib.ptr(next_done))
        if eps is None:
            self.eps.normal_()
        io = self.venv._io()
        _lib.check(self.L.rx_rollout(self.venv._h, io, r, _lib.stream_ptr(stream)), "rx_rollout")
        self.venv._launched(stream)


class StepRollout:
    """rx_rollout_steps driver: the T-step rollout of any single-agent handle as
    ONE library call that enqueues T x (rx_policy_act + rx_step) -- the kernels
    of the per-step loop, in its order, with pointer arithmetic in C instead of
    T x (tensor slicing + two ctypes calls) of host time.  The N(0, 1) noise of
    all T steps is drawn up front with ONE torch normal_() on [T, N, 2] (the
    same distribution; with T = 1 the same sample as a per-step draw); given
    the same noise every output equals the per-step loop bit for bit
    (tests/test_rollout_gpu.py)."""

    def __init__(self, agent, flat, venv, T, prec=_lib.RX_PREC_FP32):
        self.L = _lib.load()
        self.agent, self.flat, self.venv, self.T, self.prec = agent, flat, venv, int(T), int(prec)
        self.n, self.obs_dim = venv.num_envs, venv.D
        self.eps = torch.empty((self.T, self.n, 2), dtype=torch.float32, device=flat.flat_param.device)
        self._cache = {}

    @staticmethod
    def supported(venv, agent, config):
        if not hasattr(venv, "_h") or venv.n_agents != 1 or not policy_supported(agent, venv.D):
            return False
        mode = config.get("rollout_steps", "auto")
        return not (mode is False or mode == "off")

    def __call__(self, obs, actions, logprobs, dones, rewards, values, next_obs, next_done, eps=None, stream=None):
        T, n, D = self.T, self.n, self.obs_dim
        shapes = {"obs": (obs, (T, n, D)), "actions": (actions, (T, n, 2)), "logprobs": (logprobs, (T, n)),
                  "values": (values, (T, n)), "rewards": (rewards, (T, n)), "dones": (dones, (T, n)),
                  "next_obs": (next_obs, (n, D)), "next_done": (next_done, (n,))}
        e = self.eps if eps is None else eps
        key = tuple(t.data_ptr() for t in (obs, actions, logprobs, dones, rewards, values, next_obs, next_done, e))
        r = self._cache.get(key)
        if r is None:
            for k, (t, shp) in shapes.items():
                if tuple(t.shape) != shp or t.dtype != torch.float32 or not t.is_contiguous():
                    raise ValueError(f"rx_rollout_steps: {k} must be a contiguous float32 {shp}, got "
                                     f"{tuple(t.shape)} {t.dtype}")
            if tuple(e.shape) != (T, n, 2) or e.dtype != torch.float32 or not e.is_contiguous():
                raise ValueError("rx_rollout_steps: eps must be a contiguous float32 [T, N, 2]")
            if len(self._cache) > 64:
                self._cache.clear()
            r = self._cache[key] = _lib.RxRolloutIO(
                T, D, _lib.ptr(self.flat.flat_param), _lib.ptr(self.agent.log_std), _lib.ptr(e), _lib.ptr(obs),
                _lib.ptr(actions), _lib.ptr(logprobs), _lib.ptr(values), _lib.ptr(rewards), _lib.ptr(dones),
                _lib.ptr(next_obs), _lib.ptr(next_done))
        if eps is None:
            self.eps.normal_()
        io = self.venv._io()
        _lib.check(self.L.rx_rollout_steps(self.venv._h, io, r, self.prec, _lib.stream_ptr(stream)),
                   "rx_rollout_steps")
        self.venv._launched(stream)


class SelfPlayStepRollout:
    """rx_selfplay_rollout_steps driver: the self-play rollout of a two-car handle
    (rx.selfplay.SelfPlayVectorEnv with a frozen-policy opponent on
    rx_policy_act) as ONE library call enqueueing per step the opponent's and the
    agent's rx_policy_act, rx_step and one agent-row copy -- five launches where
    the per-step Python path ran nine (two noise draws, three copies).  Noise of
    both policies is drawn up front ([T, N, 2] each); given the same noise every
    output equals the per-step path bit for bit (tests/test_selfplay_train_gpu.py)."""

    def __init__(self, agent, flat, spenv, T, prec=_lib.RX_PREC_FP32):
        self.L = _lib.load()
        self.agent, self.flat, self.spenv, self.T, self.prec = agent, flat, spenv, int(T), int(prec)
        self.venv = spenv.venv
        self.n, self.obs_dim = self.venv.num_envs, self.venv.D
        dev = flat.flat_param.device
        self.eps = torch.empty((self.T, self.n, 2), dtype=torch.float32, device=dev)
        self.opp_eps = torch.empty((self.T, self.n, 2), dtype=torch.float32, device=dev)
        self.sink = torch.empty(2 * self.n, dtype=torch.float32, device=dev)
        self._cache = {}

    @staticmethod
    def supported(spenv, agent, config):
        mode = config.get("rollout_steps", "auto")
        if mode is False or mode == "off":
            return False
        v = getattr(spenv, "venv", None)
        return (v is not None and hasattr(v, "_h") and v.n_agents == 2 and spenv._opp_fused is not None
                and policy_supported(agent, v.D))

    def __call__(self, obs, actions, logprobs, dones, rewards, values, next_obs, next_done, eps=None, opp_eps=None,
                 stream=None):
        T, n, D = self.T, self.n, self.obs_dim
        e = self.eps if eps is None else eps
        oe = self.opp_eps if opp_eps is None else opp_eps
        opp = self.spenv._opp_fused
        key = tuple(t.data_ptr() for t in (obs, actions, logprobs, dones, rewards, values, next_obs, next_done, e, oe,
                                           opp.flat.flat_param, opp.agent.log_std)) + (opp.prec,)
        r = self._cache.get(key)
        if r is None:
            shapes = {"obs": (obs, (T, n, D)), "actions": (actions, (T, n, 2)), "logprobs": (logprobs, (T, n)),
                      "values": (values, (T, n)), "rewards": (rewards, (T, n)), "dones": (dones, (T, n)),
                      "next_obs": (next_obs, (n, D)), "next_done": (next_done, (n,)), "eps": (e, (T, n, 2)),
                      "opp_eps": (oe, (T, n, 2))}
            for k, (t, shp) in shapes.items():
                if tuple(t.shape) != shp or t.dtype != torch.float32 or not t.is_contiguous():
                    raise ValueError(f"rx_selfplay_rollout_steps: {k} must be a contiguous float32 {shp}")
            if len(self._cache) > 64:
                self._cache.clear()
            b = self.venv.buf
            r = self._cache[key] = (
                _lib.RxRolloutIO(T, D, _lib.ptr(self.flat.flat_param), _lib.ptr(self.agent.log_std), _lib.ptr(e),
                                 _lib.ptr(obs), _lib.ptr(actions), _lib.ptr(logprobs), _lib.ptr(values),
                                 _lib.ptr(rewards), _lib.ptr(dones), _lib.ptr(next_obs), _lib.ptr(next_done)),
                _lib.RxSelfplayIO(_lib.ptr(opp.flat.flat_param), _lib.ptr(opp.agent.log_std), _lib.ptr(oe),
                                  _lib.ptr(self.spenv._act), _lib.ptr(b["obs"]), _lib.ptr(b["reward"]),
                                  _lib.ptr(self.sink), self.spenv.agent_idx, opp.prec))
        if eps is None:
            self.eps.normal_()
        if opp_eps is None:
            self.opp_eps.normal_()
        io = self.venv._io()
        _lib.check(self.L.rx_selfplay_rollout_steps(self.venv._h, io, r[0], r[1], self.prec, _lib.stream_ptr(stream)),
                   "rx_selfplay_rollout_steps")
        self.venv._launched(stream)


# config["fused_rollout"] = "auto": the persistent rollout up to this many envs
# (one workgroup per env runs all T steps; beyond what the chip holds at once
# the workgroups would run in waves, each paying T steps of latency)
ROLLOUT_AUTO_MAX_ENVS = 256
