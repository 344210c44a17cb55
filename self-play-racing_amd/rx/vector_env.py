"""Device-resident vectorised racing envs (the host side of include/rx.h).

``RacingVectorEnv`` replaces ``gym.vector.SyncVectorEnv([RacingEnv ...])`` +
``RecordEpisodeStatistics`` (agent/ppo.py:70,85-95): every env lives as one
row of struct-of-arrays device state, and one ``rx_step`` advances all of them
(SURVEY.md §8(b)).  Two surfaces:

* device fast path -- ``reset_device`` / ``step_device`` take and return torch
  tensors on the GPU, write straight into caller buffers (e.g. the PPO rollout
  rows), and never synchronise with the host;
* SyncVectorEnv-compatible numpy surface -- ``reset`` / ``step`` return numpy
  arrays and gymnasium-style ``infos`` (``episode``/``_episode`` ...), for
  unmodified callers.

Autoreset follows gymnasium 1.x SyncVectorEnv's default NEXT_STEP mode: the
step after a terminal one ignores the action, resets the env and reports
reward 0, terminated = truncated = False (unpinned, gymnasium
is not installed here).
"""
import contextlib
import ctypes
import time

import numpy as np
import torch

from . import _lib
from .spaces import Box, single_action_space, single_observation_space
from .track import TrackSet

_AUTORESET = {"next_step": _lib.RX_AUTORESET_NEXT_STEP, "same_step": _lib.RX_AUTORESET_SAME_STEP,
              "disabled": _lib.RX_AUTORESET_DISABLED}


def _default_device():
    if not torch.cuda.is_available():
        raise _lib.RxError("RacingVectorEnv needs a HIP device (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


class _EnvProxy:
    """Stands in for ``envs.envs[i]`` (a RecordEpisodeStatistics wrapper in the
    reference).  ``setattr(envs.envs[i], 'speed_weight', w)`` (agent/ppo.py:
    256-258) lands on the wrapper there and never reaches RacingEnv (SURVEY.md
    §8 Q9), so here too it is recorded on the proxy only."""

    def __init__(self, idx):
        self.idx = idx


class _NumpyStartDraws:
    """The two-car start-slot order from the global numpy RNG, as the reference
    draws it: MultiRacingEnv.reset calls np.random.shuffle(agent_order) on a
    2-list (multi_racing_env.py:127-128), one MT19937 output u per reset (the cars
    swap when u & 1 == 0), and SyncVectorEnv resets its envs in env order.  A
    session copies the upcoming outputs to the device (from a copy of the global
    state), the launches take them in that order (rx_set_start_draws), and the
    end advances the global state by exactly the number taken."""

    def __init__(self, env):
        self.env = env
        # [used, over, stray]: rx_set_start_draws counts into the first two; a reset launched
        # between sessions (a direct rx_step / rx_reset) takes no draw and lands in [1], which
        # the next begin() stashes in [2] without a host sync -- end() reports it
        self.cursor = torch.zeros(3, dtype=torch.int64, device=env.device)
        self.buf = None
        self.active = False
        self.state0 = None

    def begin(self, cap):
        cap = max(int(cap), 1)
        self.state0 = np.random.get_state()
        u = np.random.randint(0, 2**32, size=cap, dtype=np.uint32)
        np.random.set_state(self.state0)
        if self.buf is None or self.buf.numel() < cap:
            self.buf = torch.empty(cap, dtype=torch.int32, device=self.env.device)
        self.buf[:cap].copy_(torch.from_numpy(u.view(np.int32)))
        self.cursor[2:].copy_(self.cursor[1:2])  # resets since the last session (enqueued, no sync)
        self.cursor[:2].zero_()
        _lib.check(self.env.L.rx_set_start_draws(self.env._h, _lib.ptr(self.buf), cap, _lib.ptr(self.cursor)),
                   "rx_set_start_draws")
        self.active = True

    def end(self):
        self.active = False
        torch.cuda.synchronize(self.env.device)
        used, over, stray = (int(x) for x in self.cursor.cpu().numpy())
        np.random.set_state(self.state0)
        if used:
            np.random.randint(0, 2**32, size=used, dtype=np.uint32)  # the reference's draws, consumed
        # until the next session the handle holds NO draws with a zeroed cursor: a reset
        # launched outside a session takes nothing from the buffer and is counted in
        # cursor[1]; the next session reports it.  Every count is
        # cleared here, so one report does not poison later sessions.
        self.cursor.zero_()
        _lib.check(self.env.L.rx_set_start_draws(self.env._h, _lib.ptr(self.buf), 0, _lib.ptr(self.cursor)),
                   "rx_set_start_draws")
        if over:
            raise _lib.RxError(f"start draws: {over} resets beyond the session's {self.buf.numel()} draws")
        if stray:
            raise _lib.RxError(f"start draws: {stray} resets ran outside a start-draw session (their start "
                               "slots did not come from np.random)")


def default_sort_interval(n_envs, n_agents):
    """Dynamics launches between spatial re-sorts (rx.h sort_interval) when the
    caller names none: 8 for single-agent envs above 32,768 (a re-sort is two
    launches, ~13 us at 65,536 envs, and keeps the ray waves' culling tight), 16
    elsewhere (at 4,096-16,384 envs and for two-car envs the sort costs more than
    the coherence it restores; profiles/r04/probe_sort_interval.txt)."""
    return 8 if n_agents == 1 and n_envs > 32768 else 16


class RacingVectorEnv:
    """N envs (A = 1: RacingEnv, A = 2: MultiRacingEnv) on one device.

    Parameters mirror the reference constructors: per env a control-point
    array (``track_pool[track_id]``) and a track width; ``n_sensors`` (11 in
    train.py); sensor cone pi/3 for A=1 (racing_env.py:45) and pi/2 for A=2
    (multi_racing_env.py:50).  ``sched``: launch-schedule overrides, a dict
    over ``_lib.SCHED_FIELDS`` (rx_config ABI v17: 0 = auto, -1 = off;
    scheduling only, results are identical -- the tests force each path)."""

    def __init__(self, control_points, widths, n_agents=1, n_sensors=11, device=None, autoreset="next_step",
                 seed=0, speed_weight=8.0, max_steps=3000, half_cone=None, track_set=None, cull_chunk=8,
                 sort_interval=None, ray_order=None, cull_super=8, sched=None):
        self.L = _lib.load()
        self.device = torch.device(device) if device is not None else _default_device()
        if self.device.type != "cuda":
            raise _lib.RxError(f"RacingVectorEnv runs on a HIP device, got {self.device}")
        N = len(control_points)
        if N <= 0 or len(widths) != N:
            raise ValueError("need one width per env")
        self.num_envs = N
        self.n_agents = A = int(n_agents)
        self.n_sensors = R = int(n_sensors)
        if sort_interval is None:
            sort_interval = default_sort_interval(N, A)
        self.sort_interval = int(sort_interval)
        if ray_order is None:  # direction-sorted ray tasks (rx.h ray_order 2) cover up to 16 sensors
            ray_order = 2 if R <= 16 else 1
        self.D = R + 4 + 4 * (A - 1)
        self.max_steps = int(max_steps)
        self.speed_weight = float(speed_weight)
        if half_cone is None:
            half_cone = np.pi / 3 if A == 1 else np.pi / 2
        self.tracks = track_set if track_set is not None else TrackSet()
        slots = np.empty(N, dtype=np.int32)
        cache = {}
        for i, (cp, w) in enumerate(zip(control_points, widths)):
            key = (id(cp), float(w) if w is not None else None)
            k = cache.get(key)
            if k is None:
                k = self.tracks.slot(cp, w)
                cache[key] = k
            slots[i] = k
        self.track_of_env = slots
        dev = self.device
        with torch.cuda.device(dev):
            f64 = dict(dtype=torch.float64, device=dev)
            # the bound state arrays (env order); the engine steps a working copy in
            # wave order and writes these back on demand (the `state` property)
            self._dev_newer = False
            self._last_stream = None  # stream of the last launch (state export orders after it)
            self._st = {k: torch.zeros(N * A, **f64) for k in ("x", "y", "angle", "vx", "vy", "progress",
                                                             "last_progress", "last_steering")}
            self._st["finished_step"] = torch.full((N * A,), -1, dtype=torch.int32, device=dev)
            self._st["flags"] = torch.zeros(N * A, dtype=torch.uint8, device=dev)
            self._st["steps"] = torch.zeros(N, dtype=torch.int32, device=dev)
            self._st["track"] = torch.from_numpy(slots).to(dev)
            self._st["env_flags"] = torch.zeros(N, dtype=torch.uint8, device=dev)
            self._st["ep_return"] = torch.zeros(N, **f64)
            self._st["ep_length"] = torch.zeros(N, dtype=torch.int32, device=dev)
            obs_shape = (N, self.D) if A == 1 else (N, A, self.D)
            self.buf = dict(
                actions=torch.zeros((N, A, 2), dtype=torch.float32, device=dev),
                obs=torch.zeros(obs_shape, dtype=torch.float32, device=dev),
                reward=torch.zeros((N,) if A == 1 else (N, A), dtype=torch.float32, device=dev),
                reward64=torch.zeros((N,) if A == 1 else (N, A), **f64),
                terminated=torch.zeros(N, dtype=torch.uint8, device=dev),
                truncated=torch.zeros(N, dtype=torch.uint8, device=dev),
                done_f32=torch.zeros(N, dtype=torch.float32, device=dev),
                info=torch.zeros((N, A, _lib.RX_INFO_W), **f64),
                ep_done=torch.zeros(N, dtype=torch.uint8, device=dev),
                ep_stats=torch.zeros(_lib.RX_EP_SHARDS * 4, **f64),
            )
            sched = dict(sched or {})
            bad = set(sched) - set(_lib.SCHED_FIELDS)
            if bad:
                raise ValueError(f"unknown launch-schedule keys {sorted(bad)} (known: {_lib.SCHED_FIELDS})")
            self.sched = sched
            cfg = _lib.RxConfig(N, A, R, self.max_steps, _AUTORESET[autoreset], dev.index or 0, int(seed) & (2**64 - 1),
                                float(half_cone), self.speed_weight, int(cull_chunk), self.sort_interval,
                                int(ray_order), int(cull_super), *[int(sched.get(k, 0)) for k in _lib.SCHED_FIELDS])
            h = _lib._P()
            _lib.check(self.L.rx_create(cfg, h), "rx_create")
            self._h = h
            self._upload_tracks()
            self._st["speed_weight"] = None  # per-env weights: set_speed_weights()
            st = self._state_struct()
            _lib.check(self.L.rx_bind_state(self._h, st), "rx_bind_state")
            _lib.check(self.L.rx_assign(self._h, _lib.ptr(np.ascontiguousarray(slots))), "rx_assign")
        rel = np.zeros(R, dtype=np.float64)
        _lib.check(self.L.rx_sensor_angles(self._h, _lib.ptr(rel)), "rx_sensor_angles")
        self.sensor_angles = rel
        self.single_observation_space = single_observation_space(R, A)
        self.single_action_space = single_action_space(A)
        self.observation_space = Box(-1.0, 1.0, shape=(N,) + self.single_observation_space.shape, dtype=np.float32)
        self.action_space = Box(np.tile(self.single_action_space.low, (N, 1)),
                                np.tile(self.single_action_space.high, (N, 1)), shape=(N, 2), dtype=np.float32)
        self.envs = [_EnvProxy(i) for i in range(N)]
        self.counters = None
        self._draws = None  # use_numpy_start_draws
        self._io_cache = {}
        self._episode_start = np.full(N, time.perf_counter())
        self._closed = False

    # ------------------------------------------------------------ plumbing
    def _upload_tracks(self):
        t = self.tracks.arrays()
        n = len(t["meta"])
        _lib.check(self.L.rx_upload_tracks(self._h, n, _lib.ptr(t["wp_off"]), _lib.ptr(t["wp"]), _lib.ptr(t["nrm"]),
                                           _lib.ptr(t["seg"]), _lib.ptr(t["meta"])), "rx_upload_tracks")

    def _io(self, actions=None, obs=None, reward=None, done=None, full=False):
        # per-step host cost matters (a captured 2,048-step rollout runs this
        # 2,048 times): one dict lookup when the same buffers come back
        key = (actions.data_ptr() if actions is not None else 0, obs.data_ptr() if obs is not None else 0,
               reward.data_ptr() if reward is not None else 0, done.data_ptr() if done is not None else 0, full,
               self.counters is not None)
        io = self._io_cache.get(key)
        if io is None:
            if len(self._io_cache) > 8192:
                self._io_cache.clear()
            io = self._io_cache[key] = self._make_io(actions, obs, reward, done, full)
        return io

    def _make_io(self, actions, obs, reward, done, full):
        b = self.buf
        return _lib.RxIO(
            _lib.ptr(actions) if actions is not None else None,
            _lib.ptr(obs if obs is not None else b["obs"]),
            _lib.ptr(reward if reward is not None else b["reward"]),
            _lib.ptr(b["reward64"]) if full else None,
            _lib.ptr(b["terminated"]),
            _lib.ptr(b["truncated"]),
            _lib.ptr(done if done is not None else b["done_f32"]),
            _lib.ptr(b["info"]) if full else None,
            _lib.ptr(b["ep_done"]),
            _lib.ptr(b["ep_stats"]),
            _lib.ptr(self.counters) if self.counters is not None else None,
        )

    def profile(self, mode=1):
        """rx_profile: 1 = start a fresh record of kernel durations (per-wave wall-clock
        stamps), 2 = resume recording, 0 = pause (benchmarks)."""
        _lib.check(self.L.rx_profile(self._h, int(mode)), "rx_profile")

    def profile_read(self):
        """{kernel: (mean ms, launches)} of the launches recorded since profile(True)."""
        import ctypes
        ms = (ctypes.c_double * len(_lib.RX_KERNEL_NAMES))()
        n = (ctypes.c_int32 * len(_lib.RX_KERNEL_NAMES))()
        _lib.check(self.L.rx_profile_read(self._h, ms, n), "rx_profile_read")
        return {k: (ms[i], n[i]) for i, k in enumerate(_lib.RX_KERNEL_NAMES) if n[i]}

    def profile_waves(self, launch):
        """Per-wave (start, end) device wall-clock stamps in microseconds from the
        launch's first wave start, the kernel kind name and the wave-slot count of
        recorded launch ``launch`` (rx_profile_waves; unused slots are NaN)."""
        import ctypes
        cap = self.__dict__.get("_prof_cap") or self._prof_waves_cap()
        st = np.zeros(cap, np.uint64)
        en = np.zeros(cap, np.uint64)
        n, kind, khz = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.check(self.L.rx_profile_waves(self._h, int(launch), st.ctypes.data, en.ctypes.data, cap, ctypes.byref(n),
                                           ctypes.byref(kind), ctypes.byref(khz)), "rx_profile_waves")
        m = min(n.value, cap)
        st, en = st[:m], en[:m]
        live = st > 0
        t0 = st[live].min() if live.any() else 0
        us = lambda t: np.where(live, (t.astype(np.float64) - float(t0)) * 1e3 / khz.value, np.nan)  # noqa: E731
        return us(st), us(en), _lib.RX_KERNEL_NAMES[kind.value], n.value

    def _prof_waves_cap(self):
        """Wave slots of a recorded launch (rx_profile_waves with cap 0 reports it)."""
        import ctypes
        n, kind, khz = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        z = np.zeros(1, np.uint64)
        _lib.check(self.L.rx_profile_waves(self._h, 0, z.ctypes.data, z.ctypes.data, 0, ctypes.byref(n),
                                           ctypes.byref(kind), ctypes.byref(khz)), "rx_profile_waves")
        self._prof_cap = max(1, n.value)
        return self._prof_cap

    def ray_tasks(self, stream=None):
        """The device ray-task list (rx_ray_tasks): per 64-env block its A * R task
        ids in direction-sector order, as the last sorting launch wrote it."""
        n = ctypes.c_int64(0)
        _lib.check(self.L.rx_ray_tasks(self._h, None, 0, ctypes.byref(n), None), "rx_ray_tasks")
        t = np.zeros(max(n.value, 1), np.int32)
        _lib.check(self.L.rx_ray_tasks(self._h, t.ctypes.data, n.value, ctypes.byref(n), _lib.stream_ptr(stream)),
                   "rx_ray_tasks")
        return t[:n.value]

    def ray_wave_table(self):
        """The ray-wave table in dispatch order (rx_ray_waves, host only): a dict of
        int arrays track, perm_start, task_start, count, plus per wave its class
        (the j-th 64 direction-sorted tasks of its 64-env group) and sub-wave
        (tail waves split a class's 64 tasks over ray_tail_lpr waves)."""
        n = ctypes.c_int32(0)
        _lib.check(self.L.rx_ray_waves(self._h, None, 0, ctypes.byref(n)), "rx_ray_waves")
        t = np.zeros((max(n.value, 1), 4), np.int32)
        _lib.check(self.L.rx_ray_waves(self._h, t.ctypes.data, n.value, ctypes.byref(n)), "rx_ray_waves")
        t = t[:n.value]
        off = t[:, 2].astype(np.int64) - t[:, 1].astype(np.int64) * self.n_agents * self.n_sensors
        sch = self.schedule()
        per = np.where(np.arange(len(t)) >= (sch["ray_tail_from"] if sch["ray_tail_from"] >= 0 else len(t)),
                       64 // max(1, sch["ray_tail_lpr"]), 64 // max(1, sch["ray_lpr"]))
        return {"track": t[:, 0], "perm_start": t[:, 1], "task_start": t[:, 2], "count": t[:, 3],
                "cls": np.where(t[:, 3] > 0, off // (64 // max(1, sch["ray_lpr"])), -1),
                "sub": np.where(t[:, 3] > 0, (off % 64) // per, -1)}

    def enable_counters(self, on=True):
        """Per-wave culling counters (rx_io.counters): chunk tests / scans."""
        self.counters = torch.zeros(4, dtype=torch.int64, device=self.device) if on else None

    def read_counters(self, reset=True):
        c = self.counters.cpu().numpy().copy()
        if reset:
            self.counters.zero_()
        return {"ray_chunk_tests": int(c[0]), "ray_chunks_scanned": int(c[1]), "wp_chunk_tests": int(c[2]),
                "wp_chunks_scanned": int(c[3])}

    def _state_struct(self):
        return _lib.RxState(*[_lib.ptr(self._st[k]) for k in _lib.STATE_FIELDS])

    @property
    def state(self):
        """The env state tensors in env order (x, y, angle, ... [N*A]; steps, ... [N]).
        The engine steps a working copy in wave order (rx.h, ABI v15); reading
        this property first writes it back here (rx_state_export, enqueued on
        the current stream) if a launch changed it.  After writing the tensors,
        call ``state_changed()`` (set_state does)."""
        if self._dev_newer and not self._closed:
            # export on the stream of the last launch (ordered after it), then
            # make the current stream wait for the export
            s = self._last_stream
            cur = torch.cuda.current_stream(self.device)
            _lib.check(self.L.rx_state_export(self._h, _lib.stream_ptr(s if s is not None else cur)),
                       "rx_state_export")
            if s is not None and s != cur:
                cur.wait_stream(s)
            self._dev_newer = False
        return self._st

    def state_changed(self, stream=None):
        """The state tensors were written (on ``stream``, default the current
        one): reload the engine's working copy there; the stream of the last
        launch waits for the reload, so later launches on it see the new state."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(self.L.rx_state_import(self._h, _lib.stream_ptr(s)), "rx_state_import")
        if self._last_stream is not None and self._last_stream != s:
            self._last_stream.wait_stream(s)
        self._dev_newer = False

    def _launched(self, stream=None):
        """A launch on ``stream`` (None = the current stream) changed the working state."""
        self._dev_newer = True
        self._last_stream = stream if stream is not None else torch.cuda.current_stream(self.device)

    def set_speed_weights(self, w):
        """Per-env RacingEnv.speed_weight ([N] array), or None to use the uniform value."""
        st = self.state  # current values in the bound arrays: re-binding re-reads them
        if w is None:
            st["speed_weight"] = None
        else:
            st["speed_weight"] = torch.as_tensor(np.asarray(w, dtype=np.float64).reshape(self.num_envs)).to(
                self.device).contiguous()
        torch.cuda.current_stream(self.device).synchronize()
        _lib.check(self.L.rx_bind_state(self._h, self._state_struct()), "rx_bind_state")

    def set_speed_weight(self, w):
        """RacingEnv.speed_weight for every env (racing_env.py:26,140)."""
        self.speed_weight = float(w)
        _lib.check(self.L.rx_set_speed_weight(self._h, self.speed_weight), "rx_set_speed_weight")

    def _as_actions(self, actions):
        A = self.n_agents
        if isinstance(actions, torch.Tensor):
            a = actions
            if a.dtype == torch.float32 and a.is_contiguous() and a.device == self.device and \
                    a.numel() == self.num_envs * A * 2:
                return a  # fast path: the rollout's own action rows
            if a.device != self.device or a.dtype != torch.float32:
                a = a.to(self.device, torch.float32)
        else:
            a = torch.from_numpy(np.ascontiguousarray(actions, dtype=np.float32)).to(self.device)
        if a.numel() != self.num_envs * A * 2:
            raise ValueError(f"actions must have {self.num_envs}x{A}x2 elements, got shape {tuple(a.shape)}")
        return a.contiguous()

    # ------------------------------------------------------------ start draws
    def use_numpy_start_draws(self, on=True):
        """Two-car envs: draw each reset's start-slot order from the global numpy
        RNG exactly as the reference does (np.random.shuffle in MultiRacingEnv.reset,
        multi_racing_env.py:127-128, envs in env order) instead of the device hash.
        Every reset / step / rollout then synchronises once at its end to advance
        np.random by the draws it took."""
        if self.n_agents != 2:
            raise ValueError("start-slot draws exist for two-car envs only")
        if on:
            self._draws = getattr(self, "_draws", None) or _NumpyStartDraws(self)
        else:
            self._draws = None
            _lib.check(self.L.rx_set_start_draws(self._h, None, 0, None), "rx_set_start_draws")

    @contextlib.contextmanager
    def start_draw_session(self, cap):
        """Brackets launches that may reset envs (at most ``cap`` resets in all) when
        numpy start draws are on; nested sessions join the outer one."""
        d = getattr(self, "_draws", None)
        if d is None or d.active:
            yield
            return
        d.begin(cap)
        try:
            yield
        finally:
            d.end()

    # ------------------------------------------------------------ device path
    def reset_device(self, mask=None, obs_out=None, stream=None):
        """Reset all envs (or where ``mask``, a device uint8/bool [N]); returns obs."""
        m = None
        if mask is not None:
            m = mask.to(self.device, torch.uint8).contiguous()
        io = self._io(obs=obs_out, full=True)
        with self.start_draw_session(self.num_envs):
            _lib.check(self.L.rx_reset(self._h, _lib.ptr(m), io, _lib.stream_ptr(stream)), "rx_reset")
        self._launched(stream)
        return obs_out if obs_out is not None else self.buf["obs"]

    def _step_call(self, io, phases, s):
        if phases == 3:
            _lib.check(self.L.rx_step(self._h, io, s.cuda_stream), "rx_step")
        else:
            _lib.check(self.L.rx_step_phases(self._h, io, int(phases), s.cuda_stream), "rx_step_phases")

    def step_device(self, actions, obs_out=None, reward_out=None, done_out=None, full_info=False, stream=None,
                    phases=3):
        """One step of every env from device actions; returns (obs, reward, done_f32) tensors.

        ``obs_out`` / ``reward_out`` / ``done_out`` may be rows of a rollout buffer
        (contiguous, right shape): the kernels write there directly.  ``phases``
        (rx_step_phases) splits the step into its two kernels for timing."""
        a = self._as_actions(actions)
        io = self._io(actions=a, obs=obs_out, reward=reward_out, done=done_out, full=full_info)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)  # resolved once per step
        d = self._draws
        if d is None or d.active:  # no draw session to open (the per-step host path stays short)
            self._step_call(io, phases, s)
        else:
            with self.start_draw_session(self.num_envs):
                self._step_call(io, phases, s)
        self._launched(s)
        return (obs_out if obs_out is not None else self.buf["obs"],
                reward_out if reward_out is not None else self.buf["reward"],
                done_out if done_out is not None else self.buf["done_f32"])

    def steps_device(self, actions, obs_out=None, reward_out=None, done_out=None, full_info=False, stream=None):
        """K consecutive steps from ONE call (rx_steps, ABI v21) with the actions of
        every step given up front: ``actions`` [K, N, (A,) 2] float32 on the device.
        Equal to K step_device calls on actions[0], ..., actions[K-1] bit for bit.
        ``obs_out`` / ``reward_out`` / ``done_out``: None = the env's own rows (each
        step overwrites them: they end with the last step's outputs), or [K, ...]
        buffers whose row k receives step k.  Returns the last step's (obs, reward,
        done_f32)."""
        dev_idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        on_dev = lambda t: t.is_cuda and t.device.index == dev_idx  # noqa: E731  ("cuda" == "cuda:0")
        if not isinstance(actions, torch.Tensor) or not on_dev(actions) or \
                actions.dtype != torch.float32 or not actions.is_contiguous():
            raise ValueError("steps_device takes a contiguous float32 device tensor of actions [K, N, (A,) 2]")
        A, N = self.n_agents, self.num_envs
        per = N * A * 2
        if actions.numel() % per or actions.numel() == 0:
            raise ValueError(f"actions must hold K x {N}x{A}x2 elements, got shape {tuple(actions.shape)}")
        K = actions.numel() // per
        row = {"obs": N * A * self.D, "reward": N * A, "done": N}

        def rows(t, name):
            if t is None:
                return None, 0
            if not t.is_contiguous() or not on_dev(t) or t.numel() != K * row[name]:
                raise ValueError(f"{name}_out must be a contiguous device tensor of {K} x {row[name]} elements")
            return t, row[name]

        obs_t, so = rows(obs_out, "obs")
        rew_t, sr = rows(reward_out, "reward")
        done_t, sd = rows(done_out, "done")
        io = self._io(actions=actions, obs=obs_t, reward=rew_t, done=done_t, full=full_info)
        st = _lib.RxIOStrides(actions=per, obs=so, reward=sr, done_f32=sd)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        with self.start_draw_session(K * N):
            _lib.check(self.L.rx_steps(self._h, io, int(K), ctypes.byref(st), s.cuda_stream), "rx_steps")
        self._launched(s)
        last = lambda t, n, name: self.buf[name] if t is None else t.view(K, -1)[K - 1]  # noqa: E731
        return last(obs_t, so, "obs"), last(rew_t, sr, "reward"), last(done_t, sd, "done_f32")

    def episode_stats(self, reset=True):
        """(sum of returns, sum of lengths, count) of episodes that ended since the
        last call -- one device->host copy."""
        s = self.buf["ep_stats"].view(_lib.RX_EP_SHARDS, 4).sum(0).cpu().numpy()
        if reset:
            self.buf["ep_stats"].zero_()
        return float(s[0]), float(s[1]), int(s[2])

    def env_order(self):
        """(perm, sort_bins, sort_shift): the env id at each position of the current
        wave order (diagnostics; synchronises the device)."""
        perm = np.empty(self.num_envs, np.int32)
        bins, shift = ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.check(self.L.rx_env_order(self._h, perm.ctypes.data, ctypes.byref(bins), ctypes.byref(shift)),
                   "rx_env_order")
        return perm, bins.value, shift.value

    def schedule(self):
        """The launch schedule librx resolved for this env (rx_schedule): split step,
        wide kernels, lanes per env / ray, argmin window, pre-filter, wave counts."""
        out = np.zeros(_lib.SCHEDULE_W, np.int32)
        _lib.check(self.L.rx_schedule(self._h, out.ctypes.data), "rx_schedule")
        return {k: int(v) for k, v in zip(_lib.SCHEDULE_KEYS, out)}

    def get_state(self):
        return {k: v.cpu().numpy() for k, v in self.state.items() if v is not None}

    def set_state(self, **arrays):
        """State injection (parity tests): overwrite state arrays from host arrays."""
        st = self.state
        for k, v in arrays.items():
            t = st[k]
            t.copy_(torch.as_tensor(np.ascontiguousarray(v).reshape(t.shape)).to(t.device, t.dtype))
        self.state_changed()

    # ------------------------------------------------------------ numpy surface
    def reset(self, seed=None, options=None):
        """SyncVectorEnv.reset -> every env's reset (racing_env.py:86-102)."""
        self.reset_device()
        self._episode_start[:] = time.perf_counter()
        obs = self.buf["obs"].cpu().numpy().copy()
        return obs, self._infos(reset_mask=np.ones(self.num_envs, dtype=bool), stepped=np.zeros(self.num_envs, bool))

    def step(self, actions):
        """SyncVectorEnv.step -> RecordEpisodeStatistics.step -> RacingEnv.step."""
        pending = (self.state["env_flags"] & _lib.RX_EF_PENDING_RESET).bool().cpu().numpy()
        self.step_device(actions, full_info=True)
        b = self.buf
        obs = b["obs"].cpu().numpy().copy()
        rew = b["reward64"].cpu().numpy().copy()
        term = b["terminated"].cpu().numpy().astype(bool)
        trunc = b["truncated"].cpu().numpy().astype(bool)
        infos = self._infos(reset_mask=pending, stepped=~pending, terminated=term, truncated=trunc, reward=rew)
        now = time.perf_counter()
        self._episode_start[pending] = now
        return obs, rew, term, trunc, infos

    def _infos(self, reset_mask, stepped, terminated=None, truncated=None, reward=None):
        N = self.num_envs
        st = {k: self.state[k].cpu().numpy() for k in ("x", "y", "flags")}
        inf = self.buf["info"].cpu().numpy()
        a0 = slice(0, None, self.n_agents)  # agent 0 (the learner)
        fl = st["flags"][a0]
        everyone = np.ones(N, dtype=bool)
        infos = {
            "position": np.stack([st["x"][a0], st["y"][a0]], axis=1), "_position": everyone.copy(),
            "speed": inf[:, 0, _lib.RX_INFO_SPEED].copy(), "_speed": everyone.copy(),
            "progress": inf[:, 0, _lib.RX_INFO_PROGRESS].copy(), "_progress": everyone.copy(),
            "crashed": (fl & _lib.RX_F_CRASHED) != 0, "_crashed": everyone.copy(),
            "finished": (fl & _lib.RX_F_FINISHED) != 0, "_finished": everyone.copy(),
        }
        if reward is not None and stepped.any():
            infos["reward"] = np.where(stepped, reward if reward.ndim == 1 else reward[:, 0], 0.0)
            infos["_reward"] = stepped.copy()
            if self.n_agents == 1:
                infos["progress_delta"] = np.where(stepped, inf[:, 0, _lib.RX_INFO_PROGRESS_DELTA], 0.0)
                infos["_progress_delta"] = stepped.copy()
            else:
                pl = inf[:, 0, _lib.RX_INFO_PLACEMENT].astype(np.int64)
                if (pl > 0).any():
                    infos["placement"] = pl
                    infos["_placement"] = pl > 0
        if terminated is not None:
            ended = (terminated | truncated) & stepped
            if ended.any():
                ret = self.state["ep_return"].cpu().numpy()
                ln = self.state["ep_length"].cpu().numpy()
                el = np.round(time.perf_counter() - self._episode_start, 6)
                # ep_return/ep_length were already zeroed only if reset this step;
                # ended envs are reset on the NEXT step, so their counters are intact.
                infos["episode"] = {"r": np.where(ended, ret, 0.0), "l": np.where(ended, ln, 0).astype(np.int64),
                                    "t": np.where(ended, el, 0.0)}
                infos["_episode"] = ended
        return infos

    def close(self):
        if not self._closed and getattr(self, "_h", None) is not None:
            self.L.rx_destroy(self._h)
            self._h = None
            self._closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------------------ construction helpers
    @classmethod
    def from_table(cls, path, track_of_env=None, **kw):
        """Build from an on-disk track table (rx.track.TrackSet.save): env i
        runs slot track_of_env[i] (default: the assignment stored in the file)."""
        ts, stored = TrackSet.load(path)
        toe = stored if track_of_env is None else np.asarray(track_of_env, dtype=np.int32)
        if toe is None:
            raise ValueError(f"{path} holds no env assignment: pass track_of_env")
        g = ts.geoms
        return cls([g[k].control_points for k in toe], [g[k].track_width for k in toe], track_set=ts, **kw)

    def save_table(self, path):
        """Write this env's track table and env -> slot assignment (TrackSet.save)."""
        self.tracks.save(path, self.track_of_env)

    @classmethod
    def from_envs(cls, envs, **kw):
        """Build from reference-style env objects (rx.envs.RacingEnv / MultiRacingEnv
        specs returned by a train.py ``env_fn``)."""
        envs = list(envs)
        first = envs[0]
        n_agents = getattr(first, "num_agents", 1)
        n_sensors = first.num_sensors
        for e in envs:
            if getattr(e, "num_agents", 1) != n_agents or e.num_sensors != n_sensors:
                raise ValueError("all envs of one vector env must share num_agents and num_sensors")
        cps = [e.control_points for e in envs]
        widths = [e.track_width for e in envs]
        kw.setdefault("speed_weight", getattr(first, "speed_weight", 8.0))
        return cls(cps, widths, n_agents=n_agents, n_sensors=n_sensors, **kw)
