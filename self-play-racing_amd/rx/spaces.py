"""Observation/action spaces.

Uses gymnasium.spaces when gymnasium is installed (the reference's dependency,
requirements.txt:18); otherwise a minimal Box/Dict with the members the
reference and its callers use (shape, low, high, dtype, seed, sample).
"""
import numpy as np

try:  # pragma: no cover - gymnasium is not in this image
    from gymnasium.spaces import Box, Dict  # noqa: F401
    HAVE_GYMNASIUM = True
except Exception:  # noqa: BLE001
    HAVE_GYMNASIUM = False

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            if shape is None:
                shape = np.shape(low)
            self.shape = tuple(int(s) for s in shape)
            self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()
            self._rng = np.random.default_rng()

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)
            return [seed]

        def sample(self):
            return self._rng.uniform(self.low, self.high).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Dict:
        def __init__(self, spaces):
            self.spaces = dict(spaces)

        def __getitem__(self, key):
            return self.spaces[key]

        def keys(self):
            return self.spaces.keys()

        def seed(self, seed=None):
            for i, s in enumerate(self.spaces.values()):
                s.seed(None if seed is None else seed + i)
            return [seed]


def single_action_space(n_agents=1):
    """RacingEnv / MultiRacingEnv per-agent action Box([-1, 0], [1, 1]) float32
    (racing_env.py:29-34, multi_racing_env.py:194-201)."""
    return Box(low=np.array([-1.0, 0.0]), high=np.array([1.0, 1.0]), shape=(2,), dtype=np.float32)


def single_observation_space(n_sensors=11, n_agents=1):
    """Box(-1, 1, (n_sensors + 4 + 4*(A-1),), float32) -- racing_env.py:37-42, multi_racing_env.py:204-212."""
    return Box(low=np.float32(-1.0), high=np.float32(1.0), shape=(n_sensors + 4 + 4 * (n_agents - 1),),
               dtype=np.float32)
