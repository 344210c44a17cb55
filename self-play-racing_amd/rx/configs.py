"""Hyperparameter dicts -- configs/base_config.py:1-28 and
configs/self_play_config.py:1-32 (same keys and values), plus the large-N
configurations of BASELINE.json (configs[1..4]) with their chosen horizons.
"""


def _finish(c):
    c["batch_size"] = c["num_steps"] * c["num_envs"]
    c["minibatch_size"] = c["batch_size"] // c["num_minibatches"]
    return c


def base_config(**over):
    """configs/base_config.py: single-agent PPO, 16 envs x 2048 steps."""
    c = {"total_timesteps": 5000000, "num_envs": 16, "num_steps": 2048, "learning_rate": 3e-4,
         "gamma": 0.99, "gae_lambda": 0.95, "clip_coef": 0.2, "ent_coef": 0.01, "vf_coef": 0.5,
         "update_epochs": 10, "num_minibatches": 16, "max_grad_norm": 0.5, "kl_target": 0.015,
         "seed": 1, "cuda": True, "torch_deterministic": True}
    c.update(over)
    return _finish(c)


def self_play_config(**over):
    """configs/self_play_config.py: self-play PPO, pool of 5, snapshot every 15 updates."""
    c = {"total_timesteps": 3000000, "num_envs": 16, "num_steps": 2048, "learning_rate": 3e-4,
         "gamma": 0.99, "gae_lambda": 0.97, "clip_coef": 0.2, "ent_coef": 0.02, "vf_coef": 0.5,
         "update_epochs": 10, "num_minibatches": 16, "max_grad_norm": 0.5, "kl_target": 0.015,
         "snapshot_freq": 15, "pool_size": 5, "seed": 1, "cuda": True, "torch_deterministic": True}
    c.update(over)
    return _finish(c)


# Reference naming (configs/*.py both export hyperparams_config)
hyperparams_config = base_config


def large_config(num_envs=4096, num_steps=128, **over):
    """BASELINE.json configs[1]/[2]: many envs, short horizon.  The batch is
    num_envs*num_steps; T=128 keeps the [T, N, 15] rollout at 31 MB for 4096
    envs and an update at 10 x 16 minibatches."""
    return base_config(num_envs=num_envs, num_steps=num_steps, **over)
