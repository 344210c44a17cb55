"""BASELINE.json configs[1] ("4096 parallel single-agent envs, PPO bf16"):
the policy kernels with config["policy_dtype"] = "bf16" run their products on
v_mfma_f32_16x16x32_bf16 (operands rounded to bf16, f32 accumulation).

Tolerances (stated here, derived from bf16's 8-bit significand, relative
rounding 2^-9 per operand): the forward's outputs (actions, log-probs,
values) within 2e-2 absolute of the fp32 torch forward; the minibatch
gradient within 4e-2 x max|g| per element of torch's fp32 autograd with a
cosine similarity above 0.999; one whole update's parameter change within
cosine 0.99 of the fp32 update.  The env itself is untouched by the policy
precision: replaying the bf16 rollout's recorded actions on a fresh env gives
its observations, rewards and dones bit for bit.
"""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _agent(D, seed=2, head_scale=60.0):
    from rx.agent import Agent
    from rx.spaces import Box
    torch.manual_seed(seed)
    ag = Agent(Box(-1, 1, (D,)), Box(-1, 1, (2,))).cuda()
    ag.log_std.fill_(-0.6)
    with torch.no_grad():  # non-trivial outputs (the head init is 0.01 / 1.0)
        ag.actor_mu[4].weight.mul_(head_scale)
    return ag


@pytest.mark.parametrize("D,n", [(15, 4096), (19, 300)])
def test_policy_act_bf16_close_to_torch(D, n):
    from rx import _lib
    from rx.optim import FlatAdam
    from rx.ppo_fused import PolicyAct
    ag = _agent(D)
    ref = copy.deepcopy(ag)
    fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-3, eps=1e-5), 0.5)
    pa = PolicyAct(ag, fl, n, D, _lib.RX_PREC_BF16)
    obs = torch.rand(n, D, device="cuda") * 2 - 1
    act, lp, val = (torch.empty(n, 2, device="cuda"), torch.empty(n, device="cuda"),
                    torch.empty(n, device="cuda"))
    torch.manual_seed(77)
    pa(obs, act, lp, val)
    torch.manual_seed(77)
    with torch.no_grad():
        a_ref, lp_ref, _, v_ref = ref.get_action_and_value(obs)
    assert (a_ref.abs() == 1.0).any()
    err_a = (act - a_ref).abs().max().item()
    assert err_a <= 2e-2, err_a
    assert err_a > 0  # really the bf16 path (fp32 agrees within 2e-6)
    torch.testing.assert_close(lp, lp_ref, rtol=0, atol=2e-2 * max(1.0, lp_ref.abs().max().item()))
    torch.testing.assert_close(val, v_ref.flatten(), rtol=0, atol=2e-2 * max(1.0, v_ref.abs().max().item()))


@pytest.mark.parametrize("D", [15, 19])
def test_fused_grad_bf16_close_to_autograd(D):
    from rx.optim import FlatAdam
    from rx.ppo_fused import FusedMinibatchGrad
    from tests.test_ppo_fused_gpu import _bare_ppo, _batch
    ag = _agent(D, seed=7)
    ref = copy.deepcopy(ag)
    fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-3, eps=1e-5), 0.5)
    B, mb = 4096, 1024
    b = _batch(B, D)
    perm = torch.randperm(B, device="cuda")
    p = _bare_ppo(ref)
    cfg = dict(p.config, policy_dtype="bf16")
    fg = FusedMinibatchGrad(ag, fl, b, mb, perm, cfg)
    fg.adv_stats()
    stop = torch.zeros(1, dtype=torch.bool, device="cuda")
    kl = torch.zeros(1, device="cuda")
    for m in range(B // mb):
        stop.zero_()
        fg.grad(m, stop, kl)
        ref.zero_grad()
        loss, _ = p._minibatch_loss(b, perm[m * mb:(m + 1) * mb])
        loss.backward()
        want = torch.cat([q.grad.reshape(-1) for q in ref.parameters()])
        got = fl.flat_grad
        scale = want.abs().max().item()
        err = (got - want).abs().max().item()
        cos = torch.nn.functional.cosine_similarity(got, want, dim=0).item()
        assert err <= 4e-2 * scale, (m, err, scale)
        assert cos > 0.999, (m, cos)


def test_configs1_bf16_rollout_and_update_4096_envs():
    """configs[1] end to end at its real size: 4,096 envs, a bf16 rollout (fused
    bf16 policy per step) and one bf16 update; the env outputs replay bit for bit,
    the recorded log-probs / values agree with the fp32 policy within 2e-2 (x max
    magnitude), and the bf16 update moves the parameters like the fp32 update."""
    from tests.test_ppo_gpu import _train_single_style
    from rx.vector_env import RacingVectorEnv
    N, T = 4096, 16
    tb, cfg = _train_single_style(num_envs=N, num_steps=T, policy_dtype="bf16", kl_target=1e9, update_epochs=1,
                                  num_minibatches=4)
    tf, _ = _train_single_style(num_envs=N, num_steps=T, kl_target=1e9, update_epochs=1, num_minibatches=4)
    tf.agent.load_state_dict(tb.agent.state_dict())
    bufs = tb._buffers()
    next_obs = tb.envs.buf["obs"].clone()
    next_done = torch.zeros(N, device="cuda")
    obs0 = next_obs.clone()
    out = tb.collect_rollout(*bufs, next_obs, next_done)
    obs, actions, logprobs, dones, rewards, values, next_obs, next_done, _ = out
    assert tb._fused_policy(obs) is not None and tb._fused_policy(obs).prec == 1
    # env replay: a fresh env with the same tracks, stepped with the recorded actions
    v = RacingVectorEnv.from_envs([tb.env_fn(i) for i in range(N)], device="cuda", seed=cfg["seed"])
    assert torch.equal(v.reset_device(), obs0)
    for t in range(T):
        o, r, d = v.step_device(actions[t])
        assert torch.equal(r, rewards[t]), t
        if t + 1 < T:
            assert torch.equal(o, obs[t + 1]) and torch.equal(d, dones[t + 1]), t
        else:
            assert torch.equal(o, next_obs) and torch.equal(d, next_done)
    # the bf16 policy's recorded log-probs / values vs the fp32 policy on the same obs / actions
    with torch.no_grad():
        _, lp32, _, v32 = tf.agent.get_action_and_value(obs.reshape(-1, 15), actions.reshape(-1, 2))
    torch.testing.assert_close(logprobs.reshape(-1), lp32, rtol=0, atol=2e-2 * max(1.0, lp32.abs().max().item()))
    torch.testing.assert_close(values.reshape(-1), v32.flatten(), rtol=0,
                               atol=2e-2 * max(1.0, v32.abs().max().item()))
    # one update each on the same data
    with torch.no_grad():
        nv = tb.agent.get_value(next_obs).flatten()
    adv, ret = tb.compute_advantages(rewards, dones, values, nv, next_done)
    data = [x.clone() for x in (adv, ret, values, logprobs, actions, obs)]
    before = tb._flat.flat_param.clone()
    for t in (tb, tf):
        t._anneal(0, 4)
        np.random.seed(3)
        t.ppo_update(*[x.clone() for x in data])
    d_bf = tb._flat.flat_param - before
    d_32 = tf._flat.flat_param - before
    cos = torch.nn.functional.cosine_similarity(d_bf, d_32, dim=0).item()
    assert cos > 0.99, cos
    assert float(tb._flat.step_t) == cfg["num_minibatches"] == float(tf._flat.step_t)
