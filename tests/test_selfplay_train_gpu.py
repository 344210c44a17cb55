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
