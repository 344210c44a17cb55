"""Test-only stand-in for the members of gymnasium 1.2.3 that the reference's
environment/agent modules touch at construction and step time.

gymnasium is not installed in this image (and cannot be fetched), so golden
vectors are produced by importing the reference with THIS module first on
sys.path.  Only what the reference uses is provided:

* ``Env`` -- ``reset(seed=...)`` seeds a private ``np_random`` Generator (the
  reference envs never read it), ``step`` is abstract.
* ``Wrapper`` -- attribute forwarding to ``self.env``.
* ``spaces.Box`` / ``spaces.Dict`` -- ``shape``, ``low``/``high``, ``dtype``,
  ``seed`` and ``sample`` (uniform over the box; not used by any golden vector).

Vector envs (``gymnasium.vector``) and ``wrappers.RecordEpisodeStatistics`` are
deliberately NOT provided: their autoreset/episode-statistics semantics cannot be
pinned here, and no golden vector depends on them.
"""
import numpy as np

from . import spaces  # noqa: F401


class Env:
    np_random = None

    def reset(self, *, seed=None, options=None):
        if seed is not None or self.np_random is None:
            self.np_random = np.random.default_rng(seed)
        return None

    def step(self, action):  # pragma: no cover - abstract
        raise NotImplementedError

    def close(self):
        return None


class Wrapper(Env):
    def __init__(self, env):
        self.env = env
        self.action_space = getattr(env, "action_space", None)
        self.observation_space = getattr(env, "observation_space", None)

    def __getattr__(self, name):
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def step(self, action):
        return self.env.step(action)
