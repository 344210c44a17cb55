"""Two-car self-play TRAINING at BASELINE.json configs[3]'s size (8,192 envs) on
the device path: rx.selfplay.SelfPlayPPO.train_iter (agent/self_play_ppo.py:70-187)
with the frozen-opponent rx_policy_act in the rollout.

* the pool / opponent / anneal / checkpoint cadence of 64 real updates equals
  tests/golden/schedules.npz, recorded from the reference's own
  SelfPlayPPO.train loop (snapshot every 15, pool 3, np.random.choice per update);
* pool 5 with a snapshot every update: the FIFO holds the last 5 snapshots and
  every opponent is the np.random.choice draw of a replayed generator.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_ENVS = 8192


def _selfplay(num_steps, **over):
    import random
    from rx.configs import self_play_config
    from rx.envs import MultiRacingEnv
    from rx.selfplay import SelfPlayPPO
    from rx.track import gen_tracks
    cfg = self_play_config(num_envs=N_ENVS, num_steps=num_steps, shuffle="device", checkpoint=False, **over)
    random.seed(cfg["seed"])
    np.random.seed(cfg["seed"])
    torch.manual_seed(cfg["seed"])
    pool = gen_tracks(N_ENVS, seed=cfg["seed"])
    widths = [np.random.randint(6, 10) for _ in range(N_ENVS)]
    return SelfPlayPPO(lambda i: MultiRacingEnv(2, 11, pool, i, widths), cfg, device="cuda"), cfg


def _tag(o):
    return int(round(float(o.critic[4].bias.item())))


def test_selfplay_training_cadence_matches_reference_schedule():
    """64 updates of SelfPlayPPO.train_iter at 8,192 envs (T = 4) with the
    fixture's snapshot_freq / pool_size: after each update the agent's critic
    head bias is tagged with the update index (as the fixture's generator does),
    so every snapshot names the update it was taken after.  Pool contents, the
    drawn opponent (np.random.choice), lr, log_std and the checkpoint updates
    must equal the reference's."""
    from tests.golden_util import load
    s = load("schedules.npz")
    n = int(s["selfplay_num_updates"])
    t, cfg = _selfplay(4, snapshot_freq=int(s["selfplay_snapshot_freq"]), pool_size=int(s["selfplay_pool_size"]))
    cfg["total_timesteps"] = n * cfg["batch_size"]
    np.random.seed(int(s["selfplay_np_seed"]))  # only select_opponent draws from np.random (device shuffles)
    ckpts = []
    for update, num_updates, gstep, ep, info in t.train_iter():
        assert num_updates == n
        pool = [_tag(o) for o in t.opponent_pool]
        assert pool + [-2] * (t.pool_size - len(pool)) == list(s["selfplay_pool"][update]), update
        opp = -1 if t.curr_opponent is None else _tag(t.curr_opponent)
        assert opp == s["selfplay_opponent"][update], update
        assert t.optimizer.param_groups[0]["lr"] == s["selfplay_lr"][update], update
        assert np.array_equal(t.agent.log_std.cpu().numpy(), s["selfplay_log_std"][update]), update
        assert (t.envs.opponent_policy is None) == (opp == -1)
        if t.checkpoint_due(update):
            ckpts.append(update)
        with torch.no_grad():  # tag the weights the next snapshot will copy (a view into FlatAdam's buffer)
            t.agent.critic[4].bias.fill_(float(update))
    assert ckpts == list(s["selfplay_checkpoints"])
    assert torch.isfinite(t._flat.flat_param).all()
    t.envs.close()


def test_selfplay_training_pool5_at_configs3_size():
    """configs[3]: 8,192 two-car envs, pool 5, a snapshot every update, T = 16:
    7 updates; the pool is the FIFO of the last 5 snapshots, each update's opponent
    is pool[np.random.choice(len(pool))] of a replayed generator and drives the
    rollout through the fused opponent kernel; every update takes all 160
    optimizer steps (KL stop off) and the parameters stay finite."""
    t, cfg = _selfplay(16, snapshot_freq=1, pool_size=5, kl_target=1e9)
    n = 7
    cfg["total_timesteps"] = n * cfg["batch_size"]
    np.random.seed(11)
    rep = np.random.RandomState(11)
    snaps = []
    steps0 = 0.0
    for update, num_updates, gstep, ep, info in t.train_iter():
        if update > 0:
            snaps.append(update - 1)  # the snapshot taken at this update holds the weights tagged update - 1
        want_pool = snaps[-5:]
        assert [_tag(o) for o in t.opponent_pool] == want_pool, update
        if want_pool:
            k = rep.choice(len(want_pool))
            assert _tag(t.curr_opponent) == want_pool[k], update
            assert t.envs._opp_fused is not None  # the opponent runs on rx_policy_act
        else:
            assert t.curr_opponent is None
        st = float(t._flat.step_t)
        assert st - steps0 == cfg["update_epochs"] * cfg["num_minibatches"], update
        steps0 = st
        assert gstep == (update + 1) * cfg["batch_size"]
        with torch.no_grad():
            t.agent.critic[4].bias.fill_(float(update))
    assert len(t.opponent_pool) == 5
    assert torch.isfinite(t._flat.flat_param).all()
    t.envs.close()


@pytest.mark.parametrize("n,T,prec", [(8192, 24, "fp32"), (3000, 20, "bf16")])
def test_selfplay_rollout_steps_equals_per_step_path(n, T, prec):
    """rx_selfplay_rollout_steps (ABI v19) == SelfPlayVectorEnv's per-step path
    (opponent rx_policy_act on the env's agent-1 rows, agent rx_policy_act on
    obs[t], action copy, rx_step, obs / reward copies) with the same agent and
    opponent noise, bit for bit over two chained rollouts: every buffer, the
    two-car state and the episode statistics."""
    import random
    from rx.configs import self_play_config
    from rx.envs import MultiRacingEnv
    from rx.selfplay import SelfPlayPPO
    from rx.track import gen_tracks
    res = []
    g = torch.Generator(device="cuda").manual_seed(8)
    eps = torch.randn((T, n, 2), device="cuda", generator=g) * 1.5
    oeps = torch.randn((T, n, 2), device="cuda", generator=g) * 1.5
    for fused in (True, False):
        cfg = self_play_config(num_envs=n, num_steps=T, shuffle="device", checkpoint=False, policy_dtype=prec,
                               rollout_steps="auto" if fused else False)
        random.seed(1)
        np.random.seed(1)
        torch.manual_seed(1)
        pool = gen_tracks(n, seed=1)
        widths = [np.random.randint(6, 10) for _ in range(n)]
        t = SelfPlayPPO(lambda i: MultiRacingEnv(2, 11, pool, i, widths), cfg, device="cuda")
        torch.manual_seed(5)
        t.opponent_pool.append(t.snapshot_agent())
        with torch.no_grad():  # an opponent that differs from the agent, with a visible mean
            t.opponent_pool[0].actor_mu[4].weight.mul_(40.0)
        np.random.seed(0)
        t.update_opponent()
        sp = t.envs
        bufs = t._buffers()
        nobs = sp.buf["obs"].clone()
        nd = torch.zeros(n, device="cuda")
        sr = t._step_rollout(bufs[0])
        assert (sr is not None) == fused
        for _ in range(2):
            obs, actions, logprobs, dones, rewards, values = bufs
            obs[0].copy_(nobs)
            dones[0].copy_(nd)
            if fused:
                sr(obs, actions, logprobs, dones, rewards, values, nobs, nd, eps=eps, opp_eps=oeps)
            else:
                pa = t._fused_policy(obs)
                for s in range(T):
                    pa(obs[s], actions[s], logprobs[s], values[s], eps=eps[s])
                    sp._opp_fused(sp.venv.buf["obs"][:, sp.opp_idx], sp._act[:, sp.opp_idx], eps=oeps[s])
                    sp._act[:, sp.agent_idx].copy_(actions[s])
                    last = s + 1 == T
                    o, r, _ = sp.venv.step_device(sp._act, done_out=nd if last else dones[s + 1])
                    (nobs if last else obs[s + 1]).copy_(o[:, sp.agent_idx])
                    rewards[s].copy_(r[:, sp.agent_idx])
        torch.cuda.synchronize()
        res.append(([x.clone() for x in bufs] + [nobs.clone(), nd.clone()], sp.venv.get_state(),
                    sp.venv.episode_stats()))
        sp.close()
    (ba, sa, ea), (bb, sb, eb) = res
    names = ("obs", "actions", "logprobs", "dones", "rewards", "values", "next_obs", "next_done")
    for k, x, y in zip(names, ba, bb):
        assert torch.equal(x, y), k
    assert (ba[3] > 0).any()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    assert ea[1:] == eb[1:] and ea[0] == pytest.approx(eb[0], rel=1e-12)
