"""Drop-in env classes with the reference's constructors.

``RacingEnv`` / ``MultiRacingEnv`` / ``SelfPlayWrapper`` take exactly the
arguments of environment/racing_env.py:9, multi_racing_env.py:9 and
wrappers.py:6, so a train.py ``env_fn`` works unchanged.  Constructing one is
cheap: it records the track spec (control points, width, sensors) and defers
geometry.  ``rx.ppo.PPO`` gathers the specs of all envs into ONE
``RacingVectorEnv``; used on its own, an env runs as a private 1-env device
vector env with autoreset disabled (the bare Gymnasium env contract).
"""
import numpy as np

from .spaces import Dict, single_action_space, single_observation_space
from .track import DEFAULT_CONTROL_POINTS, DEFAULT_WIDTH, TrackGeometry


def _resolve_track(track_pool, track_id, track_width):
    """Track.__init__ argument resolution -- environment/track.py:61-80."""
    if track_pool is not None:
        if track_id is None:
            track_id = np.random.randint(0, len(track_pool))  # track.py:63-64, global RNG
        cp = track_pool[track_id]
        if track_width is not None and isinstance(track_width, list):
            track_width = track_width[track_id]
    else:
        cp = DEFAULT_CONTROL_POINTS
    return cp, (DEFAULT_WIDTH if track_width is None else track_width)


class _SpecEnv:
    num_agents = 1
    half_cone = np.pi / 3

    def _init_track(self, track_pool, track_id, track_width):
        self.control_points, self.track_width = _resolve_track(track_pool, track_id, track_width)
        self._track = None
        self._venv = None

    @property
    def track(self):
        if self._track is None:
            self._track = TrackGeometry(self.control_points, self.track_width)
        return self._track

    def _vec(self):
        if self._venv is None:
            from .vector_env import RacingVectorEnv
            self._venv = RacingVectorEnv([self.control_points], [self.track_width], n_agents=self.num_agents,
                                         n_sensors=self.num_sensors, autoreset="disabled",
                                         speed_weight=getattr(self, "speed_weight", 8.0), half_cone=self.half_cone)
        return self._venv

    def close(self):
        if self._venv is not None:
            self._venv.close()
            self._venv = None


class RacingEnv(_SpecEnv):
    """environment/racing_env.py:8-167 (Gymnasium surface), device-backed."""

    metadata = {"render_modes": []}

    def __init__(self, num_sensors=7, track_pool=None, track_id=None, track_width=None, speed_weight=8.0):
        self._init_track(track_pool, track_id, track_width)
        self.num_sensors = num_sensors
        self.max_sensor_range = 50.0
        self._speed_weight = speed_weight
        self.action_space = single_action_space(1)
        self.observation_space = single_observation_space(num_sensors, 1)

    @property
    def speed_weight(self):
        return self._speed_weight

    @speed_weight.setter
    def speed_weight(self, value):
        self._speed_weight = value
        if self._venv is not None:
            self._venv.set_speed_weight(value)

    def _info(self, stepped):
        v = self._venv
        st = v.state
        inf = v.buf["info"][0, 0].cpu().numpy()
        fl = int(st["flags"][0].item())
        info = {"position": (float(st["x"][0].item()), float(st["y"][0].item())),
                "speed": float(inf[0]), "progress": float(inf[1]), "crashed": bool(fl & 1), "finished": bool(fl & 2)}
        if stepped:
            info["reward"] = float(v.buf["reward64"][0].item())
            info["progress_delta"] = float(inf[2])
        return info

    def reset(self, seed=None, options=None):
        v = self._vec()
        v.reset_device()
        return v.buf["obs"][0].cpu().numpy().copy(), self._info(False)

    def step(self, action):
        v = self._vec()
        v.step_device(np.asarray(action, dtype=np.float32).reshape(1, 2), full_info=True)
        obs = v.buf["obs"][0].cpu().numpy().copy()
        info = self._info(True)
        return (obs, info["reward"], bool(v.buf["terminated"][0].item()), bool(v.buf["truncated"][0].item()), info)


class MultiRacingEnv(_SpecEnv):
    """environment/multi_racing_env.py:8-269 (2 cars), device-backed."""

    half_cone = np.pi / 2

    def __init__(self, num_agents=2, num_sensors=11, track_pool=None, track_id=None, track_width=None):
        if num_agents != 2:
            raise NotImplementedError("the device kernel implements the 2-car race (num_agents=2) used by train.py")
        self._init_track(track_pool, track_id, track_width)
        self.num_agents = num_agents
        self.num_sensors = num_sensors
        self.max_sensor_range = 50.0
        self.speed_weight = 8.0  # read by SelfPlayWrapper.speed_weight (wrappers.py:57-63); unused by the env
        self.action_space = Dict({f"{i}": single_action_space(2) for i in range(num_agents)})
        self.observation_space = Dict({f"{i}": single_observation_space(num_sensors, 2) for i in range(num_agents)})

    def _infos(self, stepped):
        v = self._venv
        st = v.state
        inf = v.buf["info"][0].cpu().numpy()
        fl = st["flags"].cpu().numpy()
        x, y = st["x"].cpu().numpy(), st["y"].cpu().numpy()
        out = {}
        for i in range(2):
            d = {"position": (float(x[i]), float(y[i])), "speed": float(inf[i, 0]), "progress": float(inf[i, 1]),
                 "crashed": bool(fl[i] & 1), "finished": bool(fl[i] & 2)}
            if stepped:
                d["reward"] = float(v.buf["reward64"][0, i].item())
                if inf[i, 3] > 0:
                    d["placement"] = int(inf[i, 3])
            out[f"{i}"] = d
        return out

    def reset(self, seed=None, options=None):
        v = self._vec()
        v.reset_device()
        obs = v.buf["obs"][0].cpu().numpy()
        return {f"{i}": obs[i].copy() for i in range(2)}, self._infos(False)

    def step(self, actions):
        v = self._vec()
        a = np.stack([np.asarray(actions[f"{i}"], dtype=np.float32) for i in range(2)])[None]
        v.step_device(a, full_info=True)
        obs = v.buf["obs"][0].cpu().numpy()
        rew = v.buf["reward64"][0].cpu().numpy()
        term = bool(v.buf["terminated"][0].item())
        trunc = bool(v.buf["truncated"][0].item())
        dones = {f"{i}": term for i in range(2)}
        dones["__all__"] = term or trunc
        return ({f"{i}": obs[i].copy() for i in range(2)}, {f"{i}": float(rew[i]) for i in range(2)}, dones, trunc,
                self._infos(True))


class SelfPlayWrapper:
    """environment/wrappers.py:5-63: exposes agent ``agent_idx`` of a
    MultiRacingEnv; the other car is driven by ``opponent_policy`` (a frozen
    Agent) or, when None, by uniform random actions from its action space.
    Vectorised use goes through rx.selfplay.SelfPlayVectorEnv."""

    def __init__(self, env, agent_idx=0):
        self.env = env
        self.agent_idx = agent_idx
        self.opponent_idx = 1 - agent_idx
        self.action_space = env.action_space[f"{agent_idx}"]
        self.observation_space = env.observation_space[f"{agent_idx}"]
        self.opponent_policy = None
        self.opponent_action_space = env.action_space[f"{self.opponent_idx}"]
        self.last_obs_dict = None

    def set_opponent(self, opponent_policy):
        self.opponent_policy = opponent_policy

    def reset(self, **kwargs):
        obs, infos = self.env.reset(**kwargs)
        self.last_obs_dict = obs
        return obs[f"{self.agent_idx}"], infos[f"{self.agent_idx}"]

    def step(self, action):
        if self.opponent_policy is None:
            opp = self.opponent_action_space.sample()
        else:
            import torch
            p = next(self.opponent_policy.parameters())
            o = torch.from_numpy(self.last_obs_dict[f"{self.opponent_idx}"]).float().unsqueeze(0).to(p.device)
            with torch.no_grad():
                opp = self.opponent_policy.get_action_and_value(o)[0].squeeze(0).cpu().numpy()
        obs, rew, dones, trunc, infos = self.env.step({f"{self.agent_idx}": action, f"{self.opponent_idx}": opp})
        self.last_obs_dict = obs
        return (obs[f"{self.agent_idx}"], rew[f"{self.agent_idx}"], dones["__all__"], trunc,
                infos[f"{self.agent_idx}"])

    @property
    def speed_weight(self):
        return self.env.speed_weight

    @speed_weight.setter
    def speed_weight(self, value):
        self.env.speed_weight = value

    # spec passthrough for vectorisation
    @property
    def num_agents(self):
        return self.env.num_agents

    @property
    def num_sensors(self):
        return self.env.num_sensors

    @property
    def control_points(self):
        return self.env.control_points

    @property
    def track_width(self):
        return self.env.track_width
