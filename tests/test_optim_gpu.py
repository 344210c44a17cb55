"""rx_adam_clip_step (rx.optim.FlatAdam) vs torch clip_grad_norm_ + Adam
(agent/ppo.py:83,204-207), and the graph-captured PPO update vs the eager one."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _policy(seed=3):
    from rx.agent import Agent
    from rx.spaces import Box
    torch.manual_seed(seed)
    return Agent(Box(-1, 1, (15,)), Box(-1, 1, (2,))).cuda()


@pytest.mark.parametrize("max_norm", [0.5, 1e6, 0.0])
def test_flat_adam_matches_torch(max_norm):
    from rx.optim import FlatAdam
    a = _policy()
    b = copy.deepcopy(a)
    oa = torch.optim.Adam(a.parameters(), lr=3e-4, eps=1e-5)
    ob = torch.optim.Adam(b.parameters(), lr=3e-4, eps=1e-5)
    fa = FlatAdam(a, oa, max_norm)
    g = torch.Generator(device="cuda").manual_seed(0)
    for it in range(6):
        lr = 3e-4 * (1 - it / 6)
        oa.param_groups[0]["lr"] = ob.param_groups[0]["lr"] = lr
        grads = [torch.randn(p.shape, device="cuda", generator=g) * (0.1 + it) for p in b.parameters()]
        fa.zero_grad()
        for p, gr in zip(a.parameters(), grads):
            p.grad.add_(gr)  # p.grad is a view of the flat gradient buffer
        for p, gr in zip(b.parameters(), grads):
            p.grad = gr.clone()
        fa.sync_lr()
        fa.step()
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_(list(b.parameters()), max_norm)
        ob.step()
        for pa, pb in zip(a.parameters(), b.parameters()):
            torch.testing.assert_close(pa, pb, rtol=2e-5, atol=2e-7)
            torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-5, atol=1e-7)
    fa.export_state()
    sa, sb = oa.state_dict(), ob.state_dict()
    assert sa["state"].keys() == sb["state"].keys()
    for k in sa["state"]:
        assert float(sa["state"][k]["step"]) == float(sb["state"][k]["step"]) == 6.0
        torch.testing.assert_close(sa["state"][k]["exp_avg"], sb["state"][k]["exp_avg"], rtol=2e-5, atol=1e-6)
        torch.testing.assert_close(sa["state"][k]["exp_avg_sq"], sb["state"][k]["exp_avg_sq"], rtol=2e-5, atol=1e-6)


def test_flat_adam_stop_flag_and_state_roundtrip():
    from rx.optim import FlatAdam
    a = _policy()
    oa = torch.optim.Adam(a.parameters(), lr=1e-3, eps=1e-5)
    fa = FlatAdam(a, oa, 0.5)
    fa.sync_lr()
    for p in a.parameters():
        p.grad.normal_()
    fa.step()
    before = [t.clone() for t in (fa.flat_param, fa.exp_avg, fa.exp_avg_sq, fa.step_t)]
    stop = torch.ones(1, dtype=torch.bool, device="cuda")
    fa.step(stop=stop)
    for x, y in zip(before, (fa.flat_param, fa.exp_avg, fa.exp_avg_sq, fa.step_t)):
        assert torch.equal(x, y)
    # optimizer.state_dict -> fresh optimizer -> import: same flat state
    fa.export_state()
    sd = copy.deepcopy(oa.state_dict())
    c = _policy(seed=9)
    oc = torch.optim.Adam(c.parameters(), lr=1e-3, eps=1e-5)
    fc = FlatAdam(c, oc, 0.5)
    oc.load_state_dict(sd)
    fc.import_state()
    assert torch.equal(fc.exp_avg, fa.exp_avg) and torch.equal(fc.exp_avg_sq, fa.exp_avg_sq)
    assert float(fc.step_t) == 1.0
    assert [p.data_ptr() for p in c.parameters()][0] == fc.flat_param.data_ptr()


def _trainer(**over):
    from tests.test_ppo_gpu import _train_single_style
    return _train_single_style(num_envs=32, num_steps=32, **over)[0]


def _rollout(t):
    bufs = t._buffers()
    nobs = t.envs.buf["obs"].clone()
    nd = torch.zeros(t.num_local_envs, device="cuda")
    torch.manual_seed(4)
    obs, actions, logprobs, dones, rewards, values, nobs, nd, _ = t.collect_rollout(*bufs, nobs, nd)
    with torch.no_grad():
        nv = t.agent.get_value(nobs).flatten()
    adv, ret = t.compute_advantages(rewards, dones, values, nv, nd)
    return adv, ret, values, logprobs, actions, obs


@pytest.mark.parametrize("kl_target", [1e9, 2e-4])
def test_graph_update_equals_eager_update(kl_target, capsys):
    """Graph-captured epochs (device KL flag) == eager minibatch loop with the
    reference's immediate return: same parameters, Adam state and np.random state."""
    res = []
    for graph in (True, False):
        t = _trainer(graph_update=graph, fused_update=False, kl_target=kl_target)
        data = _rollout(t)
        np.random.seed(123)
        for u in range(2):
            t._anneal(u, 4)
            t.ppo_update(*data)
        res.append(([p.detach().clone() for p in t.agent.parameters()], t._flat.exp_avg.clone(),
                     float(t._flat.step_t), np.random.get_state()[1].copy(), np.random.get_state()[2]))
    (pa, ma, sa, ra, pa_pos), (pb, mb, sb, rb, pb_pos) = res
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)
    assert torch.equal(ma, mb) and sa == sb
    assert np.array_equal(ra, rb) and pa_pos == pb_pos
    if kl_target < 1:
        assert 0 < sa < 2 * 10 * 16  # stopped early somewhere
        assert "Early stopping" in capsys.readouterr().out


def test_flat_update_close_to_torch_adam():
    """The flat-optimizer update follows torch.optim.Adam + clip_grad_norm_ within float rounding
    (one optimizer step: later Adam steps amplify last-bit gradient differences of near-zero
    components into +-lr moves, which would test Adam's conditioning, not the kernel)."""
    over = dict(kl_target=1e9, update_epochs=1, num_minibatches=1)
    ta = _trainer(graph_update=False, **over)
    tb = _trainer(**over)
    tb.agent.load_state_dict(ta.agent.state_dict())
    tb._flat = None  # reference torch.optim path
    data = _rollout(ta)
    np.random.seed(5)
    ta.ppo_update(*data)
    np.random.seed(5)
    tb.ppo_update(*data)
    for x, y in zip(ta.agent.parameters(), tb.agent.parameters()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-6)
