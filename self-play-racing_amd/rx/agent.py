"""Actor-critic policy -- agent/ppo.py:11-62, same modules, init and state_dict
keys (actor_mu.{0,2,4}, critic.{0,2,4}, log_std buffer), so checkpoints move
between the reference and this engine unchanged (SURVEY.md §5 checkpoint row).

This module is the parameter container and the torch reference forward.  On
the default device path the MLP does NOT run on rocBLAS: the rollout's
forward + sampling is the hand-written MFMA kernel k_policy_act
(rx.ppo_fused.PolicyAct, rx_ppo.hip) and the PPO minibatch forward / loss /
backward is k_ppo_grad (v_mfma_f32_16x16x4_f32, or the bf16 MFMA with
config["policy_dtype"] = "bf16"), both over the flat parameter buffer that
backs these modules' tensors (rx.optim.FlatAdam).  The torch forward here
(get_action_and_value) is what config["fused_policy"] / ["fused_update"] =
False fall back to, and what the parity tests compare the kernels against.
"""
import numpy as np
import torch
import torch.nn as nn


class Agent(nn.Module):
    def __init__(self, obs_space, action_space):
        super().__init__()
        obs_dim = int(np.array(obs_space.shape).prod())
        act_dim = action_space.shape[0]
        lin = Agent.layer_optimization
        # mean head bounded by tanh; the std is a fixed (annealed) buffer, not a parameter
        self.actor_mu = nn.Sequential(lin(nn.Linear(obs_dim, 64)), nn.Tanh(), lin(nn.Linear(64, 64)), nn.Tanh(),
                                      lin(nn.Linear(64, act_dim), std=0.01), nn.Tanh())
        self.register_buffer("log_std", torch.zeros(act_dim))
        self.critic = nn.Sequential(lin(nn.Linear(obs_dim, 64)), nn.Tanh(), lin(nn.Linear(64, 64)), nn.Tanh(),
                                    lin(nn.Linear(64, 1), std=1.0))

    def get_value(self, obs):
        return self.critic(obs)

    def get_action_and_value(self, obs, action=None):
        """Sample (or score) an action: Normal(mu, exp(log_std)); samples are
        clamped to [-1, 1] and the log-prob is of the CLAMPED action (SURVEY.md
        §8 Q7), summed over the 2 action dims; entropy likewise."""
        mu = self.actor_mu(obs).float()  # no-op in fp32; under bf16 autocast only the GEMMs are bf16
        # validate_args=False: the default check is a host sync (illegal inside a
        # captured rollout); scale = exp(log_std) > 0 always, so only NaN inputs
        # would behave differently (no ValueError)
        std = torch.exp(self.log_std).expand_as(mu)
        dist = torch.distributions.Normal(mu, std, validate_args=False)
        if action is None:
            with torch.no_grad():
                # = dist.sample() = torch.normal(mu, std) bit for bit (ATen normal_out_impl
                # draws N(0, 1) into the output, then mul_(std).add_(mean)) without its
                # std.min() >= 0 host check, which cannot run inside a captured graph
                eps = torch.empty_like(mu).normal_()
                action = torch.clamp(eps.mul_(std).add_(mu), -1.0, 1.0)
        return action, dist.log_prob(action).sum(-1), dist.entropy().sum(-1), self.critic(obs).float()

    @staticmethod
    def layer_optimization(layer, std=np.sqrt(2), bias=0.0):
        torch.nn.init.orthogonal_(layer.weight, std)
        torch.nn.init.constant_(layer.bias, bias)
        return layer
