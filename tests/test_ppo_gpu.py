"""PPO drop-in (rx.ppo) on the device env: reference train.py wiring, rollout
semantics of agent/ppo.py:97-132, GAE/update plumbing."""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train_single_style(num_envs=32, num_steps=16, updates=2, **over):
    """train.py:65-115 with rx imports (the drop-in)."""
    from rx.configs import base_config
    from rx.envs import RacingEnv
    from rx.ppo import PPO
    from rx.track import gen_tracks
    config = base_config(num_envs=num_envs, num_steps=num_steps, **over)
    config["total_timesteps"] = updates * config["batch_size"]
    random.seed(config["seed"])
    np.random.seed(config["seed"])
    torch.manual_seed(config["seed"])
    pool = gen_tracks(num_tracks=config["num_envs"], seed=config["seed"])
    widths = [np.random.randint(6, 10) for _ in range(config["num_envs"])]

    def env_fn(env_idx):
        return RacingEnv(num_sensors=11, track_pool=pool, track_id=env_idx, track_width=widths[env_idx])

    return PPO(env_fn, config, device="cuda"), config


def test_train_single_dropin_runs(tmp_path):
    trainer, config = _train_single_style()
    trainer.info_path = str(tmp_path / "info.json")
    info = trainer.train()
    assert isinstance(info, dict) and "rewards" in info
    p = tmp_path / "m.pth"
    trainer.save(str(p))
    sd = torch.load(str(p), weights_only=True)
    assert sorted(sd.keys())[0].startswith("actor_mu")
    trainer.load(str(p))


def test_collect_rollout_equals_reference_loop():
    """The zero-copy rollout (env writes into obs[t+1]/rewards[t]/dones[t+1])
    produces exactly the buffers of the reference's copy-per-step loop."""
    t1, c = _train_single_style(num_envs=64, num_steps=24, fused_policy=False)
    t2, _ = _train_single_style(num_envs=64, num_steps=24)
    t2.agent.load_state_dict(t1.agent.state_dict())
    bufs1 = t1._buffers()
    nobs1 = t1.envs.buf["obs"].clone()
    nd1 = torch.zeros(64, device="cuda")
    torch.manual_seed(11)
    out1 = t1.collect_rollout(*bufs1, nobs1, nd1)
    # reference-style loop on the twin env
    obs, actions, logprobs, dones, rewards, values = t2._buffers()
    next_obs = t2.envs.buf["obs"].clone()
    next_done = torch.zeros(64, device="cuda")
    torch.manual_seed(11)
    with torch.no_grad():
        for step in range(c["num_steps"]):
            obs[step].copy_(next_obs)
            dones[step].copy_(next_done)
            a, lp, _, v = t2.agent.get_action_and_value(next_obs)
            actions[step].copy_(a)
            logprobs[step].copy_(lp)
            values[step].copy_(v.flatten())
            o, r, d = t2.envs.step_device(a)
            rewards[step].copy_(r)
            next_obs.copy_(o)
            next_done.copy_(d)
    for x, y in zip(out1[:8], (obs, actions, logprobs, dones, rewards, values, next_obs, next_done)):
        assert torch.equal(x, y)


def test_agent_sampling_is_torch_normal():
    """Agent's capture-safe sampling == Normal(mu, std).sample() (agent/ppo.py:56) bit for bit."""
    from rx.agent import Agent
    from rx.spaces import Box
    torch.manual_seed(3)
    ag = Agent(Box(-1, 1, (11,)), Box(-1, 1, (2,))).cuda()
    ag.log_std.fill_(-0.7)
    obs = torch.randn(1000, 11, device="cuda")
    torch.manual_seed(5)
    a, lp, ent, v = ag.get_action_and_value(obs)
    torch.manual_seed(5)
    with torch.no_grad():
        mu = ag.actor_mu(obs)
        d = torch.distributions.Normal(mu, torch.exp(ag.log_std).expand_as(mu))
        ref = torch.clamp(d.sample(), -1.0, 1.0)
    assert torch.equal(a, ref)
    assert torch.equal(lp, d.log_prob(ref).sum(-1)) and torch.equal(ent, d.entropy().sum(-1))


@pytest.mark.parametrize("fused_rollout", ["auto", False])
def test_graph_rollout_equals_eager_across_updates(fused_rollout):
    """The captured rollout replays with the CURRENT weights, log_std and RNG
    state: two updates with graph_rollout on == the same two updates eager
    (persistent k_rollout, and the per-step policy + rx_step path)."""
    outs = []
    for graph in (True, False):
        t, c = _train_single_style(num_envs=64, num_steps=16, graph_rollout=graph, fused_rollout=fused_rollout)
        bufs = t._buffers()
        nobs = t.envs.buf["obs"].clone()
        nd = torch.zeros(64, device="cuda")
        seq = []
        for u in range(2):
            t._anneal(u, 4)
            out = t.collect_rollout(*bufs, nobs, nd)
            obs, actions, logprobs, dones, rewards, values, nobs, nd, ep = out
            seq.append([x.clone() for x in out[:8]])
            with torch.no_grad():
                nv = t.agent.get_value(nobs).flatten()
            adv, ret = t.compute_advantages(rewards, dones, values, nv, nd)
            t.ppo_update(adv, ret, values, logprobs, actions, obs)
            # the env state read back after a replay must be the replayed one (not a
            # stale export): ADVICE r02, graph replays mark the working state newer
            seq.append([torch.from_numpy(v) for _, v in sorted(t.envs.get_state().items())])
        outs.append(seq)
    for ua, ub in zip(*outs):
        for x, y in zip(ua, ub):
            assert torch.equal(x, y)


def test_selfplay_graph_rollout_equals_eager():
    """Self-play (configs[3]'s wiring, frozen pool opponent): the captured rollout
    (graph_rollout = True) == the eager one over two rollouts, buffers and the
    two-car env state bit for bit."""
    from rx.configs import self_play_config
    from rx.envs import MultiRacingEnv
    from rx.selfplay import SelfPlayPPO
    from rx.track import gen_tracks
    outs = []
    for graph in (True, False):
        config = self_play_config(num_envs=64, num_steps=16, graph_rollout=graph)
        random.seed(1)
        np.random.seed(1)
        torch.manual_seed(1)
        pool = gen_tracks(num_tracks=64, seed=1)
        widths = [np.random.randint(6, 10) for _ in range(64)]
        t = SelfPlayPPO(lambda i: MultiRacingEnv(2, 11, pool, i, widths), config, device="cuda")
        t.opponent_pool.append(t.snapshot_agent())
        t.update_opponent()
        bufs = t._buffers()
        nobs = t.envs.buf["obs"].clone()
        nd = torch.zeros(64, device="cuda")
        seq = []
        for _ in range(2):
            out = t.collect_rollout(*bufs, nobs, nd)
            nobs, nd = out[6], out[7]
            seq.append([x.clone() for x in out[:8]])
            seq.append([torch.from_numpy(v) for _, v in sorted(t.envs.venv.get_state().items())])
        outs.append(seq)
    for ua, ub in zip(*outs):
        for x, y in zip(ua, ub):
            assert torch.equal(x, y)


def test_gae_in_ppo_is_reference_formula():
    trainer, c = _train_single_style(num_envs=16, num_steps=8)
    g = torch.Generator(device="cuda").manual_seed(0)
    T, N = 8, 16
    r = torch.randn(T, N, device="cuda", generator=g)
    v = torch.randn(T, N, device="cuda", generator=g)
    d = (torch.rand(T, N, device="cuda", generator=g) < 0.2).float()
    nv = torch.randn(N, device="cuda", generator=g)
    nd = torch.rand(N, device="cuda", generator=g) < 0.2
    adv, ret = trainer.compute_advantages(r, d, v, nv, nd)
    # agent/ppo.py:134-154 verbatim on the same device
    A = torch.zeros_like(r)
    run = 0
    for t in reversed(range(T)):
        if t == T - 1:
            nnt = 1.0 - nd.to(torch.float32)
            nvt = nv
        else:
            nnt = 1.0 - d[t + 1]
            nvt = v[t + 1]
        delta = r[t] + (c["gamma"] * nnt * nvt) - v[t]
        A[t] = run = delta + c["gamma"] * c["gae_lambda"] * nnt * run
    assert torch.equal(adv, A) and torch.equal(ret, A + v)


def test_train_multi_dropin_runs(tmp_path):
    """train.py:16-63 (self-play) with rx imports, tiny budget: snapshots, pool, checkpoint."""
    from rx.configs import self_play_config
    from rx.envs import MultiRacingEnv
    from rx.selfplay import SelfPlayPPO
    from rx.track import gen_tracks
    config = self_play_config(num_envs=32, num_steps=8, snapshot_freq=2, pool_size=2)
    config["total_timesteps"] = 12 * config["batch_size"]
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    pool = gen_tracks(num_tracks=32, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(32)]

    def env_fn(i):
        return MultiRacingEnv(num_agents=2, num_sensors=11, track_pool=pool, track_id=i, track_width=widths)

    t = SelfPlayPPO(env_fn, config, device="cuda")
    t.info_path = str(tmp_path / "sp.json")
    t.checkpoint_fmt = str(tmp_path / "ck_{}.pth")
    info = t.train()
    assert len(t.opponent_pool) == 2  # snapshots at updates 2,4,...,10, FIFO of 2
    ck = tmp_path / "ck_10.pth"
    assert ck.exists()
    u, gs, inf = t.load_checkpoint(str(ck))
    assert u == 10 and gs == 11 * config["batch_size"]
    assert "opponent_pool_size" in info


def test_selfplay_opponent_batched_forward():
    from rx.agent import Agent
    from rx.selfplay import SelfPlayVectorEnv
    from rx.track import gen_tracks
    from rx.vector_env import RacingVectorEnv
    np.random.seed(1)
    pool = gen_tracks(8, seed=1)
    v = RacingVectorEnv(pool, [7] * 8, n_agents=2, device="cuda")
    sp = SelfPlayVectorEnv(v)
    obs = sp.reset_device()
    assert obs.shape == (8, 19)
    opp = Agent(v.single_observation_space, v.single_action_space).cuda()
    sp.set_opponent(opp)
    a = torch.zeros(8, 2, device="cuda")
    o, r, d = sp.step_device(a)
    assert o.shape == (8, 19) and r.shape == (8,) and d.shape == (8,)
    assert torch.equal(sp._act[:, 0], a) and sp._act[:, 1].abs().max() <= 1.0


def test_evaluator_protocol_runs():
    from rx.agent import Agent
    from rx.evaluate import Evaluator
    ev = Evaluator(max_steps=300, device="cuda")
    assert ev.venv.num_envs == 200 and len(ev.venv.tracks) <= 12
    torch.manual_seed(0)
    ag = Agent(ev.venv.single_observation_space, ev.venv.single_action_space).cuda()
    res = ev.run(ag)
    assert res["num_episodes"] == 200 and 0.0 <= res["success_rate"] <= 1.0
    assert res["crash_rate"] > 0.5  # an untrained policy crashes
    ev.close()


def test_multi_evaluator_protocol_runs():
    """evaluate_multi_agent_overall on the device: 200 two-car episodes, both cars
    driven by the policy, reference summary keys + per-episode list."""
    from rx.agent import Agent
    from rx.evaluate import MultiEvaluator
    ev = MultiEvaluator(max_steps=200, device="cuda")
    assert ev.venv.num_envs == 200 and ev.venv.n_agents == 2
    torch.manual_seed(0)
    ag = Agent(ev.venv.single_observation_space, ev.venv.single_action_space).cuda()
    res = ev.run(ag)
    assert res["num_episodes"] == 200 and 0.0 <= res["success_rate"] <= 1.0
    assert len(res["all_episodes"]) == 200 and "placement" in res["all_episodes"][0]
    assert all(1 <= e["steps"] <= 200 for e in res["all_episodes"])
    ev.close()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_next_value_matches_critic_and_draws_no_rng(dtype):
    """GAE's bootstrap value on the fused policy path (PPO._next_value, round 5):
    the rx_policy_act critic -- the kernel that computed the rollout's values --
    within float rounding of agent.get_value (bf16: its matrix-core tolerance),
    with no draw from torch's CUDA generator (the rollout noise stream is the
    reference's), and torch's forward when config fused_next_value is off."""
    t, _ = _train_single_style(num_envs=64, num_steps=8, policy_dtype=dtype)
    g = torch.Generator(device="cuda").manual_seed(3)
    obs = torch.rand((64, 15), device="cuda", generator=g) * 2 - 1
    with torch.no_grad():
        want = t.agent.get_value(obs).flatten()
    state = torch.cuda.get_rng_state()
    with torch.no_grad():
        got = t._next_value(obs).clone()
    torch.cuda.synchronize()
    assert torch.equal(state, torch.cuda.get_rng_state())
    tol = 2e-5 if dtype == "fp32" else 3e-2
    torch.testing.assert_close(got, want, rtol=tol, atol=tol * float(want.abs().max()))
    # the same kernel, the same floats, as the rollout's value rows
    pa = t._fused_policy(obs.unsqueeze(0))
    act, val = torch.empty((64, 2), device="cuda"), torch.empty(64, device="cuda")
    pa(obs, act, None, val, eps=torch.zeros((64, 2), device="cuda"))
    assert torch.equal(val, got)
    t.config["fused_next_value"] = False
    with torch.no_grad():
        assert torch.equal(t._next_value(obs), want)
