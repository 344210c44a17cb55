"""Agent (agent/ppo.py:11-62) parity on CPU: init, state_dict layout, forward."""
import numpy as np
import torch


def _box(shape):
    from rx.spaces import Box
    return Box(-1.0, 1.0, shape=shape, dtype=np.float32)


def test_agent_matches_reference_init_and_forward(golden):
    from rx.agent import Agent
    g = golden["agent"]
    for d in (15, 19):
        torch.manual_seed(1)
        ag = Agent(_box((d,)), _box((2,)))
        ag.log_std.fill_(-0.5)
        sd = ag.state_dict()
        ref_keys = sorted(k[len(f"d{d}_sd_"):] for k in g.files if k.startswith(f"d{d}_sd_"))
        assert sorted(sd.keys()) == ref_keys
        for k in ref_keys:
            assert np.array_equal(sd[k].numpy(), g[f"d{d}_sd_{k}"]), k
        obs = torch.from_numpy(g[f"d{d}_obs"])
        act = torch.from_numpy(g[f"d{d}_act"])
        with torch.no_grad():
            _, logp, ent, val = ag.get_action_and_value(obs, act)
            mu = ag.actor_mu(obs)
        assert np.array_equal(mu.numpy(), g[f"d{d}_mu"])
        assert np.array_equal(logp.numpy(), g[f"d{d}_logp"])
        assert np.array_equal(ent.numpy(), g[f"d{d}_ent"])
        assert np.array_equal(val.numpy(), g[f"d{d}_val"])
        n_params = sum(p.numel() for p in ag.parameters())
        assert n_params == (10563 if d == 15 else 11075)


def test_sampled_actions_are_clamped():
    from rx.agent import Agent
    torch.manual_seed(0)
    ag = Agent(_box((15,)), _box((2,)))
    ag.log_std.fill_(1.0)
    a, logp, ent, v = ag.get_action_and_value(torch.zeros(4096, 15))
    assert a.abs().max() <= 1.0 and v.shape == (4096, 1) and logp.shape == (4096,)
