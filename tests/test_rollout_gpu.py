"""Persistent small-N rollout (rx_rollout / k_rollout) == the per-step fused
rollout (rx_policy_act + rx_step, agent/ppo.py:97-132) bit for bit, given the
same N(0, 1) noise: observations, actions, log-probs, values, rewards, dones,
the env state and the episode statistics."""
import numpy as np
import pytest
import torch

from tests.test_ppo_gpu import _train_single_style

pytestmark = pytest.mark.gpu


def _per_step(t, eps, obs, actions, logprobs, dones, rewards, values, next_obs, next_done):
    """The fused per-step path with injected noise: rx_policy_act on eps[t], then rx_step."""
    from rx import _lib
    L = _lib.load()
    T, n, D = obs.shape
    for s in range(T):
        io = _lib.RxPolicyIO(D, n, _lib.ptr(obs[s]), _lib.ptr(eps[s]), _lib.ptr(t._flat.flat_param),
                             _lib.ptr(t.agent.log_std), _lib.ptr(actions[s]), _lib.ptr(logprobs[s]),
                             _lib.ptr(values[s]), 0, 0)
        _lib.check(L.rx_policy_act(io, _lib.stream_ptr()), "rx_policy_act")
        last = s + 1 == T
        t.envs.step_device(actions[s], obs_out=next_obs if last else obs[s + 1], reward_out=rewards[s],
                           done_out=next_done if last else dones[s + 1])


@pytest.mark.parametrize("n,T", [(16, 400), (200, 160), (1, 2048)])
def test_rollout_equals_per_step_path(n, T):
    ta, c = _train_single_style(num_envs=n, num_steps=T)
    tb, _ = _train_single_style(num_envs=n, num_steps=T)
    tb.agent.load_state_dict(ta.agent.state_dict())
    from rx.ppo_fused import Rollout
    assert Rollout.supported(ta.envs, ta.agent, c)
    ro = ta._fused_rollout(T)
    assert ro is not None
    g = torch.Generator(device="cuda").manual_seed(4)
    eps = torch.randn((T, n, 2), device="cuda", generator=g) * 1.5  # wide noise: crashes, resets, clamps
    outs = []
    for tr, fused in ((ta, True), (tb, False)):
        bufs = tr._buffers()
        nobs = tr.envs.buf["obs"].clone()
        nd = torch.zeros(n, device="cuda")
        for _ in range(2):  # two rollouts: the second starts from mid-episode state
            obs, actions, logprobs, dones, rewards, values = bufs
            obs[0].copy_(nobs)
            dones[0].copy_(nd)
            if fused:
                ro(obs, actions, logprobs, dones, rewards, values, nobs, nd, eps=eps)
            else:
                _per_step(tr, eps, obs, actions, logprobs, dones, rewards, values, nobs, nd)
        torch.cuda.synchronize()
        outs.append(([x.clone() for x in bufs] + [nobs.clone(), nd.clone()], tr.envs.get_state(),
                     tr.envs.episode_stats()))
    (ba, sa, ea), (bb, sb, eb) = outs
    names = ("obs", "actions", "logprobs", "dones", "rewards", "values", "next_obs", "next_done")
    for k, x, y in zip(names, ba, bb):
        assert torch.equal(x, y), k
    assert (ba[3] > 0).any(), "no episode ended: the autoreset path was not exercised"
    assert (ba[1].abs() == 1.0).any()  # clamped samples
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    assert ea[1:] == eb[1:] and ea[0] == pytest.approx(eb[0], rel=1e-12)


@pytest.mark.parametrize("autoreset", ["same_step", "disabled"])
def test_rollout_other_autoreset_modes(autoreset):
    """k_rollout's one-kernel branch (same-step autoreset: dyn1_env FULL before
    the raycast) and the split branch with autoreset disabled, each == the
    per-step path on a twin env, bit for bit."""
    from rx.agent import Agent
    from rx.optim import FlatAdam
    from rx.ppo_fused import Rollout
    from rx.spaces import Box
    from rx.vector_env import RacingVectorEnv
    from rx.track import gen_tracks
    n, T = 24, 300
    pool = gen_tracks(num_tracks=n, seed=3)
    widths = [6 + (i % 4) for i in range(n)]
    torch.manual_seed(9)
    ag = Agent(Box(-1, 1, (15,)), Box(-1, 1, (2,))).cuda()
    ag.log_std.fill_(-0.3)
    fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-3, eps=1e-5), 0.5)
    g = torch.Generator(device="cuda").manual_seed(6)
    eps = torch.randn((T, n, 2), device="cuda", generator=g) * 1.5
    outs = []
    for fused in (True, False):
        venv = RacingVectorEnv(pool, widths, device="cuda", autoreset=autoreset)
        obs = torch.zeros((T, n, 15), device="cuda")
        actions = torch.zeros((T, n, 2), device="cuda")
        logprobs, dones, rewards, values = (torch.zeros((T, n), device="cuda") for _ in range(4))
        nobs = venv.reset_device().clone()
        nd = torch.zeros(n, device="cuda")
        obs[0].copy_(nobs)
        dones[0].copy_(nd)
        if fused:
            Rollout(ag, fl, venv, T)(obs, actions, logprobs, dones, rewards, values, nobs, nd, eps=eps)
        else:
            class _T:  # the attributes _per_step reads
                pass
            tr = _T()
            tr._flat, tr.agent, tr.envs = fl, ag, venv
            _per_step(tr, eps, obs, actions, logprobs, dones, rewards, values, nobs, nd)
        torch.cuda.synchronize()
        outs.append(([x.clone() for x in (obs, actions, logprobs, dones, rewards, values, nobs, nd)],
                     venv.get_state()))
        venv.close()
    (ba, sa), (bb, sb) = outs
    for k, x, y in zip(("obs", "actions", "logprobs", "dones", "rewards", "values", "next_obs", "next_done"), ba, bb):
        assert torch.equal(x, y), k
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    if autoreset == "same_step":
        assert (ba[3] > 0).any(), "no episode ended: the reset path was not exercised"


def test_rollout_used_by_collect_rollout_and_trains():
    """collect_rollout takes the persistent path for few envs (config
    "fused_rollout" auto) and a short train() runs on it."""
    t, c = _train_single_style(num_envs=16, num_steps=64)
    assert t._fused_rollout(64) is not None
    t2, _ = _train_single_style(num_envs=16, num_steps=64, fused_rollout=False)
    assert t2._fused_rollout(64) is None
    bufs = t._buffers()
    nobs = t.envs.buf["obs"].clone()
    nd = torch.zeros(16, device="cuda")
    out = t.collect_rollout(*bufs, nobs, nd)
    assert torch.isfinite(out[2]).all() and torch.isfinite(out[5]).all()
    assert out[1].abs().max() <= 1.0


def test_configs0_one_env_ppo_iteration():
    """configs[0] ("1 env, from-scratch PPO"): one PPO iteration at num_envs = 1,
    num_steps = 2048 (configs/base_config.py:5-27 otherwise) on the HIP path --
    the rollout as ONE k_rollout workgroup (== the per-step path bit for bit:
    test_rollout_equals_per_step_path[1-2048]), GAE, then 10 epochs x 16
    minibatches of 128 rows through k_ppo_grad (graph-captured epochs) -- and
    the same update on the same batch through the torch path (fused_policy =
    fused_update = False: torch autograd + the flat Adam), agent/ppo.py:97-209.
    Equal optimizer-step counts and np.random consumption; parameters within the
    G8 float32 tolerance (tests/test_ppo_golden.py).  KL early stop off so a
    borderline KL cannot split the two runs."""
    T = 2048
    ta, c = _train_single_style(num_envs=1, num_steps=T, kl_target=1e9)
    tb, _ = _train_single_style(num_envs=1, num_steps=T, kl_target=1e9, fused_policy=False, fused_update=False)
    tb.agent.load_state_dict(ta.agent.state_dict())
    assert ta._fused_rollout(T) is not None and tb._fused_rollout(T) is None
    assert c["minibatch_size"] == 128
    bufs = ta._buffers()
    nobs = ta.envs.buf["obs"].clone()
    nd = torch.zeros(1, device="cuda")
    obs, actions, logprobs, dones, rewards, values, nobs, nd, ep = ta.collect_rollout(*bufs, nobs, nd)
    assert float(dones.sum()) > 0, "no episode ended in 2,048 steps"
    with torch.no_grad():
        nv = ta.agent.get_value(nobs).flatten()
    adv, ret = ta.compute_advantages(rewards, dones, values, nv, nd)
    batch = [x.clone() for x in (adv, ret, values, logprobs, actions, obs)]
    np.random.seed(123)
    ta.ppo_update(*batch)
    rng_a = np.random.get_state()
    np.random.seed(123)
    tb.ppo_update(*[x.clone() for x in batch])
    rng_b = np.random.get_state()
    torch.cuda.synchronize()
    assert np.array_equal(rng_a[1], rng_b[1]) and rng_a[2] == rng_b[2]
    n = int(float(ta._flat.step_t))
    assert n == int(float(tb._flat.step_t)) == 160
    lr = c["learning_rate"]
    sa, sb = ta.agent.state_dict(), tb.agent.state_dict()
    for k in sa:
        np.testing.assert_allclose(sa[k].cpu().numpy(), sb[k].cpu().numpy(), rtol=1e-4, atol=0.02 * lr * n,
                                   err_msg=k)


@pytest.mark.parametrize("n,T,prec", [(4096, 64, "fp32"), (4096, 32, "bf16"), (3000, 40, "bf16"), (64, 30, "fp32")])
def test_rollout_steps_equals_per_step_path(n, T, prec):
    """rx_rollout_steps (ABI v19: T x (rx_policy_act + rx_step) enqueued by ONE
    call, the default eager rollout of every single-agent handle the persistent
    kernel does not take) == the Python per-step loop bit for bit with the same
    noise -- configs[1]'s 4,096 envs (split step, 4 lanes per ray), a ragged
    3,000 in bf16, and 64 envs on the small-N kernels -- over two chained
    rollouts: every buffer, the env state and the episode statistics."""
    ta, c = _train_single_style(num_envs=n, num_steps=T, policy_dtype=prec, fused_rollout=False)
    tb, _ = _train_single_style(num_envs=n, num_steps=T, policy_dtype=prec, fused_rollout=False)
    tb.agent.load_state_dict(ta.agent.state_dict())
    bufs_a = ta._buffers()
    sr = ta._step_rollout(bufs_a[0])
    assert sr is not None and sr.prec == (1 if prec == "bf16" else 0)
    g = torch.Generator(device="cuda").manual_seed(6)
    eps = torch.randn((T, n, 2), device="cuda", generator=g) * 1.5
    outs = []
    for tr, fused in ((ta, True), (tb, False)):
        bufs = tr._buffers()
        nobs = tr.envs.buf["obs"].clone()
        nd = torch.zeros(n, device="cuda")
        for _ in range(2):
            obs, actions, logprobs, dones, rewards, values = bufs
            obs[0].copy_(nobs)
            dones[0].copy_(nd)
            if fused:
                sr(obs, actions, logprobs, dones, rewards, values, nobs, nd, eps=eps)
            else:
                pa = tr._fused_policy(obs)
                for s in range(T):
                    pa(obs[s], actions[s], logprobs[s], values[s], eps=eps[s])
                    last = s + 1 == T
                    tr.envs.step_device(actions[s], obs_out=nobs if last else obs[s + 1], reward_out=rewards[s],
                                        done_out=nd if last else dones[s + 1])
        torch.cuda.synchronize()
        outs.append(([x.clone() for x in bufs] + [nobs.clone(), nd.clone()], tr.envs.get_state(),
                     tr.envs.episode_stats()))
    (ba, sa, ea), (bb, sb, eb) = outs
    names = ("obs", "actions", "logprobs", "dones", "rewards", "values", "next_obs", "next_done")
    for k, x, y in zip(names, ba, bb):
        assert torch.equal(x, y), k
    assert (ba[3] > 0).any() and (ba[1].abs() == 1.0).any()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    assert ea[1:] == eb[1:] and ea[0] == pytest.approx(eb[0], rel=1e-12)


def test_collect_rollout_uses_rollout_steps_and_keeps_t1_stream():
    """collect_rollout takes rx_rollout_steps for configs[1]-size handles; with
    T = 1 its [1, N, 2] noise draw is the very sample a per-step [N, 2] draw
    makes, so the step equals the per-step fused path run from the same seed."""
    ta, _ = _train_single_style(num_envs=4096, num_steps=1)
    tb, _ = _train_single_style(num_envs=4096, num_steps=1, rollout_steps=False)
    tb.agent.load_state_dict(ta.agent.state_dict())
    outs = []
    for t in (ta, tb):
        bufs = t._buffers()
        nobs = t.envs.buf["obs"].clone()
        nd = torch.zeros(4096, device="cuda")
        torch.manual_seed(3)
        outs.append(t.collect_rollout(*bufs, nobs, nd))
    assert ta.__dict__.get("_steps_rollout") is not None and tb.__dict__.get("_steps_rollout") is None
    for x, y in zip(outs[0][:8], outs[1][:8]):
        assert torch.equal(x, y)
