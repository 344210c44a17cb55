"""rx_random_permutation (ABI v16): the device minibatch shuffle of
PPO.ppo_update for config shuffle = "device" (the reference shuffles b_inds
with np.random.shuffle on the host, agent/ppo.py:165-171; that default path
is pinned bit for bit by tests/test_ppo_golden.py).  Checked here: the output
is a permutation of 0 .. n-1 for awkward n, the seed keys it, and the first
entry is spread evenly over a small n."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _perm(n, seed):
    from rx import _lib
    L = _lib.load()
    out = torch.full((max(n, 1),), -1, dtype=torch.int64, device="cuda")
    _lib.check(L.rx_random_permutation(n, seed, _lib.ptr(out), _lib.stream_ptr(None)), "rx_random_permutation")
    torch.cuda.synchronize()
    return out[:n].cpu().numpy()


@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000, 32768, 524288, (1 << 20) + 7])
def test_is_a_permutation(n):
    p = _perm(n, 12345)
    assert np.array_equal(np.sort(p), np.arange(n))


def test_seed_keys_the_permutation():
    a, b, c = _perm(4096, 1), _perm(4096, 1), _perm(4096, 2)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, c)
    assert (a != np.arange(4096)).mean() > 0.99  # not near the identity


def test_first_entry_is_spread_evenly():
    n, trials = 8, 4000
    first = np.array([_perm(n, s)[0] for s in range(trials)])
    counts = np.bincount(first, minlength=n)
    chi2 = float(((counts - trials / n) ** 2 / (trials / n)).sum())
    assert chi2 < 40.0, counts  # 7 degrees of freedom: p ~ 1e-6 at 40


def test_ppo_device_shuffle_uses_it(monkeypatch):
    """config shuffle = "device": every epoch's row order comes from
    rx_random_permutation (no torch.randperm / rocprim sort)."""
    from rx import _lib
    calls = []
    L = _lib.load()
    real = L.rx_random_permutation

    def spy(n, seed, out, stream):
        calls.append(int(n))
        return real(n, seed, out, stream)

    from rx.configs import base_config
    from rx.envs import RacingEnv
    from rx.ppo import PPO
    from rx.track import gen_tracks
    np.random.seed(1)
    pool = gen_tracks(64, seed=1)
    cfg = base_config(num_envs=64, num_steps=32, shuffle="device", kl_target=1e9)
    p = PPO(lambda i: RacingEnv(11, pool, i, 8), cfg)
    monkeypatch.setattr(L, "rx_random_permutation", spy)
    bufs = p._buffers()
    nobs = p.envs.buf["obs"].clone()
    nd = torch.zeros(p.num_local_envs, device="cuda")
    obs, actions, logprobs, dones, rewards, values, nobs, nd, _ = p.collect_rollout(*bufs, nobs, nd)
    with torch.no_grad():
        nv = p.agent.get_value(nobs).flatten()
    adv, ret = p.compute_advantages(rewards, dones, values, nv, nd)
    p.ppo_update(adv, ret, values, logprobs, actions, obs)
    assert calls == [64 * 32] * cfg["update_epochs"]


@pytest.mark.gpu
@pytest.mark.parametrize("kl_target", [1e9, 0.02, 0.004, 1e-5])
def test_async_epochs_equal_per_epoch_sync(kl_target, capsys):
    """Device shuffles enqueue every epoch without a host KL check in between
    (rx.ppo.PPO._update_epochs_async); parameters, Adam state, step count, the
    early-stop message and torch's CPU generator must end exactly as with the
    synchronous per-epoch check (config["epoch_sync"] = True)."""
    from rx.configs import base_config
    from rx.envs import RacingEnv
    from rx.ppo import PPO
    from rx.track import gen_tracks
    out = {}
    for sync in (True, False):
        np.random.seed(1)
        pool = gen_tracks(64, seed=1)
        cfg = base_config(num_envs=64, num_steps=32, shuffle="device", kl_target=kl_target, epoch_sync=sync)
        p = PPO(lambda i: RacingEnv(11, pool, i, 8), cfg)
        bufs = p._buffers()
        nobs = p.envs.buf["obs"].clone()
        nd = torch.zeros(p.num_local_envs, device="cuda")
        obs, actions, logprobs, dones, rewards, values, nobs, nd, _ = p.collect_rollout(*bufs, nobs, nd)
        with torch.no_grad():
            nv = p.agent.get_value(nobs).flatten()
        adv, ret = p.compute_advantages(rewards, dones, values, nv, nd)
        capsys.readouterr()
        p.ppo_update(adv, ret, values, logprobs, actions, obs)
        torch.cuda.synchronize()
        f = p._flat
        out[sync] = (f.flat_param.clone(), f.exp_avg.clone(), f.exp_avg_sq.clone(), float(f.step_t.item()),
                     torch.get_rng_state().clone(), capsys.readouterr().out)
        p.envs.close()
    a, b = out[True], out[False]
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    assert a[3] == b[3]
    assert torch.equal(a[4], b[4])
    assert a[5] == b[5]
    if kl_target < 1e-4:
        assert "Early stopping" in a[5]
