"""Fused PPO minibatch gradient (rx_ppo_minibatch_grad) vs torch autograd of
the reference loss (agent/ppo.py:170-203), and the fused update's control flow."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bare_ppo(agent, **over):
    from rx.configs import base_config
    from rx.ppo import PPO
    p = PPO.__new__(PPO)
    p.config = base_config(**over)
    p.device = torch.device("cuda")
    p.agent = agent
    return p


def _batch(B, D, seed=0, adv_scale=5.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    obs = torch.rand(B, D, generator=g, device="cuda") * 2 - 1
    act = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
    logp = torch.randn(B, generator=g, device="cuda") * 0.3 - 1.0
    adv = torch.randn(B, generator=g, device="cuda") * adv_scale + 0.3
    ret = torch.randn(B, generator=g, device="cuda") * 10
    val = ret + torch.randn(B, generator=g, device="cuda") * 0.3  # some value-clip ties / both branches
    return obs, act, logp, adv, ret, val


@pytest.mark.parametrize("D", [15, 19])
def test_fused_grad_matches_autograd(D):
    from rx.agent import Agent
    from rx.optim import FlatAdam
    from rx.ppo_fused import FusedMinibatchGrad, supported
    from rx.spaces import Box
    torch.manual_seed(7)
    ag = Agent(Box(-1, 1, (D,)), Box(-1, 1, (2,))).cuda()
    ag.log_std.fill_(-0.8)
    with torch.no_grad():  # non-trivial outputs (the head init is 0.01 / 1.0)
        ag.actor_mu[4].weight.mul_(60.0)
    ref = copy.deepcopy(ag)
    fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-3, eps=1e-5), 0.5)
    B, mb = 2048, 512
    b = _batch(B, D)
    b_ppo = (b[0], b[1], b[2], b[3], b[4], b[5])
    perm = torch.randperm(B, device="cuda")
    assert supported(ag, b_ppo, mb)
    cfg = _bare_ppo(ref).config
    fg = FusedMinibatchGrad(ag, fl, b_ppo, mb, perm, cfg)
    fg.adv_stats()
    stop = torch.zeros(1, dtype=torch.bool, device="cuda")
    kl = torch.zeros(1, device="cuda")
    p = _bare_ppo(ref)
    # the PPO loss on (obs, act, logp, adv, ret, val) in _minibatch_loss order
    bt = (b[0], b[1], b[2], b[3], b[4], b[5])
    for m in range(B // mb):
        stop.zero_()
        fg.grad(m, stop, kl)
        ref.zero_grad()
        loss, akl = p._minibatch_loss(bt, perm[m * mb:(m + 1) * mb])
        loss.backward()
        want = torch.cat([q.grad.reshape(-1) for q in ref.parameters()])
        got = fl.flat_grad
        scale = want.abs().max()
        torch.testing.assert_close(got, want, rtol=2e-4, atol=2e-5 * float(scale))
        assert bool(stop) == (float(akl) > cfg["kl_target"])  # random old log-probs: KL is large
        # kl: the fused kernel accumulates in double; compare to torch's mean
        s = float(fg.ws_d.sum()) / mb  # one KL partial per workgroup
        assert abs(s - float(akl)) <= 1e-5 + 1e-4 * abs(float(akl))


def _trainer(**over):
    from tests.test_ppo_gpu import _train_single_style
    return _train_single_style(num_envs=32, num_steps=32, **over)[0]


def _rollout(t):
    from tests.test_optim_gpu import _rollout as r
    return r(t)


def test_fused_update_step_close_to_torch():
    """One fused optimizer step == one torch autograd + flat Adam step within float rounding."""
    over = dict(kl_target=1e9, update_epochs=1, num_minibatches=1)
    ta = _trainer(**over)                      # graph + fused
    tb = _trainer(graph_update=False, **over)  # eager autograd, flat Adam
    tb.agent.load_state_dict(ta.agent.state_dict())
    data = _rollout(ta)
    np.random.seed(5)
    ta.ppo_update(*data)
    np.random.seed(5)
    tb.ppo_update(*data)
    assert next(iter(ta._upd_graphs.values())).fused is not None
    torch.testing.assert_close(ta._flat.flat_grad, tb._flat.flat_grad, rtol=2e-4,
                               atol=2e-5 * float(tb._flat.flat_grad.abs().max()))
    for x, y in zip(ta.agent.parameters(), tb.agent.parameters()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=2e-6)


def test_fused_update_early_stop_and_full_run(capsys):
    t = _trainer(kl_target=-1.0)  # every KL exceeds it: stop at the first minibatch
    data = _rollout(t)
    before = t._flat.flat_param.clone()
    np.random.seed(9)
    st = np.random.get_state()
    t._anneal(0, 4)
    t.ppo_update(*data)
    after = np.random.get_state()
    assert torch.equal(before, t._flat.flat_param) and float(t._flat.step_t) == 0.0
    assert "Early stopping at epoch 1" in capsys.readouterr().out
    np.random.set_state(st)
    np.random.shuffle(np.arange(32 * 32))  # exactly one shuffle consumed, as the reference's return
    now = np.random.get_state()
    assert np.array_equal(now[1], after[1]) and now[2] == after[2]
    t2 = _trainer(kl_target=1e9)
    data2 = _rollout(t2)
    t2._anneal(0, 4)
    t2.ppo_update(*data2)
    c = t2.config
    assert float(t2._flat.step_t) == c["update_epochs"] * (c["batch_size"] // c["minibatch_size"])
    assert not torch.equal(t2._flat.flat_param, before)


@pytest.mark.parametrize("D,n", [(15, 16), (15, 4100), (19, 300)])
def test_policy_act_matches_torch(D, n):
    """rx_policy_act == get_action_and_value (agent/ppo.py:48-59) on the same N(0,1)
    draw: actions / log-probs / values within float rounding."""
    from rx.agent import Agent
    from rx.optim import FlatAdam
    from rx.ppo_fused import PolicyAct
    from rx.spaces import Box
    torch.manual_seed(2)
    ag = Agent(Box(-1, 1, (D,)), Box(-1, 1, (2,))).cuda()
    ag.log_std.fill_(-0.6)
    with torch.no_grad():
        ag.actor_mu[4].weight.mul_(80.0)  # mu spread over (-1, 1), some clamped samples
    ref = copy.deepcopy(ag)
    fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-3, eps=1e-5), 0.5)
    pa = PolicyAct(ag, fl, n, D)
    obs = torch.rand(n, D, device="cuda") * 2 - 1
    act = torch.empty(n, 2, device="cuda")
    lp = torch.empty(n, device="cuda")
    val = torch.empty(n, device="cuda")
    torch.manual_seed(77)
    pa(obs, act, lp, val)
    torch.manual_seed(77)
    with torch.no_grad():
        a_ref, lp_ref, _, v_ref = ref.get_action_and_value(obs)
    assert (a_ref.abs() == 1.0).any()  # the clamp is exercised
    torch.testing.assert_close(act, a_ref, rtol=0, atol=2e-6)
    torch.testing.assert_close(lp, lp_ref, rtol=1e-5, atol=5e-5)
    torch.testing.assert_close(val, v_ref.flatten(), rtol=1e-5, atol=1e-5)


def test_policy_act_near_zero_preactivations():
    """tanh_fast near 0 (rx_policy.h): with every weight scaled down the hidden
    pre-activations are ~1e-5, where 1 - 2/(exp(2|x|) + 1) alone would cancel to a
    relative error of ~6e-3; the small-|x| select keeps the policy within float
    rounding RELATIVE to its tiny outputs.  log_std = -20 makes the action ~ mu.
    Tolerance: 2e-5 relative to each output's scale (float rounding of a 64-term sum;
    without the select the error is ~6e-3 of it)."""
    from rx.agent import Agent
    from rx.optim import FlatAdam
    from rx.ppo_fused import PolicyAct
    from rx.spaces import Box
    torch.manual_seed(4)
    D, n = 15, 512
    ag = Agent(Box(-1, 1, (D,)), Box(-1, 1, (2,))).cuda()
    ag.log_std.fill_(-20.0)
    with torch.no_grad():
        for seq in (ag.actor_mu, ag.critic):
            seq[0].weight.mul_(1e-5)
        ag.actor_mu[4].weight.mul_(100.0)  # mu ~ 1e-5 rather than 1e-7
    ref = copy.deepcopy(ag)
    fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-3, eps=1e-5), 0.5)
    pa = PolicyAct(ag, fl, n, D)
    obs = torch.rand(n, D, device="cuda") * 2 - 1
    act = torch.empty(n, 2, device="cuda")
    lp = torch.empty(n, device="cuda")
    val = torch.empty(n, device="cuda")
    torch.manual_seed(78)
    pa(obs, act, lp, val)
    torch.manual_seed(78)
    with torch.no_grad():
        a_ref, _, _, v_ref = ref.get_action_and_value(obs)
    v_ref = v_ref.flatten()
    assert 1e-7 < float(v_ref.abs().median()) < 1e-3 and 1e-7 < float(a_ref.abs().median()) < 1e-3
    # relative to the outputs' own scale (a row whose sum cancels has no relative bound)
    torch.testing.assert_close(val, v_ref, rtol=2e-5, atol=2e-5 * float(v_ref.abs().max()))
    torch.testing.assert_close(act, a_ref, rtol=2e-5, atol=2e-5 * float(a_ref.abs().max()))


def test_fused_policy_rollout_runs_and_differs_only_by_rounding():
    """A fused-policy rollout step == the torch-policy step on the same state and noise
    (first step only: later steps may diverge chaotically through crash thresholds)."""
    from tests.test_ppo_gpu import _train_single_style
    ta, c = _train_single_style(num_envs=64, num_steps=1)
    tb, _ = _train_single_style(num_envs=64, num_steps=1, fused_policy=False)
    tb.agent.load_state_dict(ta.agent.state_dict())
    outs = []
    for t in (ta, tb):
        bufs = t._buffers()
        nobs = t.envs.buf["obs"].clone()
        nd = torch.zeros(64, device="cuda")
        torch.manual_seed(3)
        outs.append(t.collect_rollout(*bufs, nobs, nd))
    for x, y in zip(outs[0][:6], outs[1][:6]):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=5e-5)


def test_selfplay_fused_opponent_matches_torch_opponent():
    """SelfPlayVectorEnv with the frozen opponent on rx_policy_act (strided two-car
    obs read in place, actions written into the [N, 2, 2] buffer) == the torch
    forward of the same opponent on the same N(0, 1) draw, within rounding."""
    from rx.agent import Agent
    from rx.optim import FlatParams
    from rx.selfplay import SelfPlayVectorEnv
    from rx.track import gen_tracks
    from rx.vector_env import RacingVectorEnv
    np.random.seed(1)
    pool = gen_tracks(4, seed=1)
    N = 300
    v = RacingVectorEnv([pool[i % 4] for i in range(N)], [7] * N, n_agents=2, device="cuda")
    sp = SelfPlayVectorEnv(v)
    sp.reset_device()
    torch.manual_seed(0)
    opp = Agent(v.single_observation_space, v.single_action_space).cuda()
    opp.log_std.fill_(-0.5)
    with torch.no_grad():
        opp.actor_mu[4].weight.mul_(50.0)
    ref = copy.deepcopy(opp)
    sp.set_opponent(opp, FlatParams(opp))
    assert sp._opp_fused is not None
    torch.manual_seed(9)
    sp._opponent_actions()
    got = sp._act[:, 1].clone()
    torch.manual_seed(9)
    with torch.no_grad():
        want = ref.get_action_and_value(v.buf["obs"][:, 1])[0]
    torch.testing.assert_close(got, want, rtol=0, atol=2e-6)
    assert torch.equal(sp._act[:, 0], torch.zeros_like(sp._act[:, 0]))  # agent 0's slot untouched


def test_fused_update_graph_equals_eager():
    """The fused update replayed from captured epoch graphs == the same launches issued eagerly."""
    res = []
    for graph in (True, False):
        t = _trainer(graph_update=graph, kl_target=1e9)
        data = _rollout(t)
        np.random.seed(4)
        for u in range(2):
            t._anneal(u, 4)
            t.ppo_update(*data)
        ent = next(iter(t._upd_graphs.values()))
        assert ent.fused is not None and (ent.graph is not None) == graph
        res.append((t._flat.flat_param.clone(), t._flat.exp_avg_sq.clone(), float(t._flat.step_t)))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1]) and res[0][2] == res[1][2]


@pytest.mark.parametrize("kl_target", [1e9, -1.0])
def test_shard_update_world1_equals_fused(kl_target):
    """The data-parallel launch sequence (adv moments -> finalize, shard grad
    scaled by 1/world with the KL in the bucket slot, rx_ppo_kl_check, Adam) at
    world = 1 == the single-rank fused update bit for bit, early stop included."""
    res = []
    for shard in (False, True):
        t = _trainer(graph_update=False, shard_update=shard, kl_target=kl_target)
        data = _rollout(t)
        np.random.seed(4)
        for u in range(2):
            t._anneal(u, 4)
            t.ppo_update(*data)
        res.append((t._flat.flat_param.clone(), t._flat.exp_avg.clone(), float(t._flat.step_t)))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1]) and res[0][2] == res[1][2]
    if kl_target < 0:
        assert res[0][2] == 0.0


def test_adv_moments_finalize_equals_adv_stats():
    """rx_ppo_adv_moments -> rx_ppo_adv_finalize(count = mb) == rx_ppo_adv_stats bit for bit;
    with moments summed over two shards, finalize matches float64 statistics of the union."""
    from rx import _lib
    L = _lib.load()
    B, mb, D = 4096, 512, 15
    obs, act, logp, adv, ret, val = _batch(B, D, seed=3)
    perm = torch.randperm(B, device="cuda")
    params = torch.zeros(L.rx_ppo_n_params(D), device="cuda")
    log_std = torch.zeros(2, device="cuda")
    stats = torch.zeros(2 * (B // mb), device="cuda")
    b = _lib.RxPPOBatch(D, mb, B, *[_lib.ptr(t) for t in (obs, act, logp, adv, ret, val, perm, params, log_std,
                                                           stats)], 0.2, 0.5, 0.015)
    s = _lib.stream_ptr()
    _lib.check(L.rx_ppo_adv_stats(b, B // mb, _lib.ptr(stats), s))
    mom = torch.zeros((B // mb, 2), dtype=torch.float64, device="cuda")
    st2 = torch.zeros_like(stats)
    _lib.check(L.rx_ppo_adv_moments(b, B // mb, _lib.ptr(mom), s))
    _lib.check(L.rx_ppo_adv_finalize(_lib.ptr(mom), B // mb, mb, _lib.ptr(st2), s))
    assert torch.equal(stats, st2)
    # two shards of half-minibatches: moments add, finalize over 2 * (mb / 2) rows
    half = _lib.RxPPOBatch(D, mb // 2, B, *[_lib.ptr(t) for t in (obs, act, logp, adv, ret, val, perm, params,
                                                                   log_std, stats)], 0.2, 0.5, 0.015)
    m2 = torch.zeros((2 * (B // mb), 2), dtype=torch.float64, device="cuda")
    _lib.check(L.rx_ppo_adv_moments(half, 2 * (B // mb), _lib.ptr(m2), s))
    summed = (m2[0::2] + m2[1::2]).contiguous()  # minibatch m = half-minibatches 2m and 2m+1
    st3 = torch.zeros_like(stats)
    _lib.check(L.rx_ppo_adv_finalize(_lib.ptr(summed), B // mb, mb, _lib.ptr(st3), s))
    a = adv.double()[perm].view(B // mb, mb)
    ref = torch.stack([a.mean(1), a.std(1)], 1).reshape(-1).float()
    torch.testing.assert_close(st3, ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("B,mb", [(4096, 512), (524288, 32768), (2048, 128)])
def test_adv_stats_ws_spread_over_workgroups(B, mb):
    """rx_ppo_adv_stats_ws (ABI v17: 2,048-row chunks on their own workgroups,
    then a fold in chunk order): == float64 statistics of each minibatch of the
    permuted advantages within float32 rounding (agent/ppo.py:186-187), and its
    moments -> rx_ppo_adv_finalize(count = mb) == its stats bit for bit."""
    from rx import _lib
    L = _lib.load()
    D = 15
    obs, act, logp, adv, ret, val = _batch(B, D, seed=5)
    perm = torch.randperm(B, device="cuda")
    params = torch.zeros(L.rx_ppo_n_params(D), device="cuda")
    log_std = torch.zeros(2, device="cuda")
    n_mb = B // mb
    stats = torch.zeros(2 * n_mb, device="cuda")
    b = _lib.RxPPOBatch(D, mb, B, *[_lib.ptr(t) for t in (obs, act, logp, adv, ret, val, perm, params, log_std,
                                                           stats)], 0.2, 0.5, 0.015)
    ws = torch.empty(L.rx_ppo_adv_workspace_doubles(mb, n_mb), dtype=torch.float64, device="cuda")
    assert ws.numel() == 2 * n_mb * max(1, mb // 2048)
    s = _lib.stream_ptr()
    _lib.check(L.rx_ppo_adv_stats_ws(b, n_mb, _lib.ptr(ws), _lib.ptr(stats), None, s), "adv_stats_ws")
    a = adv.double()[perm].view(n_mb, mb)
    ref = torch.stack([a.mean(1), a.std(1)], 1).reshape(-1).float()
    torch.testing.assert_close(stats, ref, rtol=1e-6, atol=1e-6)
    mom = torch.zeros((n_mb, 2), dtype=torch.float64, device="cuda")
    _lib.check(L.rx_ppo_adv_stats_ws(b, n_mb, _lib.ptr(ws), None, _lib.ptr(mom), s), "adv_moments_ws")
    st2 = torch.zeros_like(stats)
    _lib.check(L.rx_ppo_adv_finalize(_lib.ptr(mom), n_mb, mb, _lib.ptr(st2), s), "finalize")
    assert torch.equal(stats, st2)
