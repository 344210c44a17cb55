"""C-ABI library: builds, loads without a GPU and exports every include/rx.h symbol."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "rx.h")).read()
    return sorted(set(re.findall(r"^(?:const\s+)?\w+\s*\*?\s*(rx_\w+)\s*\(", src, re.M)))


def test_header_declares_the_abi():
    names = _declared()
    for n in ("rx_create", "rx_destroy", "rx_upload_tracks", "rx_assign", "rx_bind_state", "rx_reset", "rx_step",
              "rx_gae", "rx_gae_scan", "rx_last_error", "rx_sensor_angles"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from rx import _build
    path = _build.build(verbose=False)
    lib = ctypes.CDLL(path)
    for n in _declared():
        assert hasattr(lib, n), n
    lib.rx_abi_version.restype = ctypes.c_int
    from rx._lib import ABI_VERSION
    assert lib.rx_abi_version() == ABI_VERSION


def test_create_without_device_fails_loudly():
    from rx import _lib
    L = _lib.load()
    cfg = _lib.RxConfig(16, 1, 11, 3000, 0, 0, 0, 1.0471975511965976, 8.0)
    h = _lib._P()
    rc = L.rx_create(cfg, h)
    import torch
    if not torch.cuda.is_available():
        assert rc != 0 and L.rx_last_error()
    else:  # pragma: no cover - GPU box
        assert rc == 0
        L.rx_destroy(h)
    bad = _lib.RxConfig(16, 3, 11, 3000, 0, 0, 0, 1.0, 8.0)
    assert L.rx_create(bad, h) == _lib.RX_EINVAL
    assert b"n_agents" in L.rx_last_error()


def test_update_abi_validates_without_device():
    """The PPO-update / policy entry points check their arguments before any HIP call."""
    import ctypes
    from rx import _lib
    L = _lib.load()
    assert L.rx_ppo_n_params(15) == 10563 and L.rx_ppo_n_params(19) == 11075 and L.rx_ppo_n_params(7) == 0
    assert L.rx_ppo_workspace_floats(15, 32768) % 64 == 0 and L.rx_ppo_workspace_doubles(32768) >= 1
    assert L.rx_ppo_workspace_floats(3, 64) == 0
    b = _lib.RxPPOBatch()
    b.obs_dim, b.mb, b.n_rows = 11, 64, 128
    assert L.rx_ppo_adv_stats(ctypes.byref(b), 2, None, None) == _lib.RX_EINVAL
    assert b"obs_dim" in L.rx_last_error()
    b.obs_dim = 15
    assert L.rx_ppo_minibatch_grad(ctypes.byref(b), 0, None, None, None, None, None, None) == _lib.RX_EINVAL
    assert b"null" in L.rx_last_error()
    io = _lib.RxPolicyIO()
    io.obs_dim, io.n = 15, 4
    assert L.rx_policy_act(ctypes.byref(io), None) == _lib.RX_EINVAL
    # persistent rollout: null handle / buffers are rejected before any HIP call
    assert L.rx_rollout_supported(None) == 0
    r = _lib.RxRolloutIO()
    r.T, r.obs_dim = 8, 15
    assert L.rx_rollout(None, ctypes.byref(_lib.RxIO()), ctypes.byref(r), None) == _lib.RX_EINVAL
    assert b"null" in L.rx_last_error()
    cfg = _lib.RxAdamConfig()
    cfg.n_tensors = 0
    assert L.rx_adam_clip_step(ctypes.byref(cfg), None, None, None, None, None, None, None, None, None) \
        == _lib.RX_EINVAL
    assert b"n_tensors" in L.rx_last_error()
    assert L.rx_adam_workspace_floats(ctypes.byref(cfg)) == 0
    cfg.n_tensors, cfg.beta1, cfg.beta2 = 2, 0.9, 0.999
    cfg.offsets[1], cfg.offsets[2] = 1000, 2050
    assert L.rx_adam_workspace_floats(ctypes.byref(cfg)) == 33 * 2 + 2  # ceil(2050 / 64) norm blocks x 2 tensors + 2 scalars
    # fused minibatch update (ABI v13): argument checks before any launch
    assert L.rx_ppo_update_workspace_floats(15, ctypes.byref(cfg)) > 0
    assert L.rx_ppo_update_workspace_floats(7, ctypes.byref(cfg)) == 0
    b.obs_dim = 15
    args = [None] * 12
    assert L.rx_ppo_minibatch_update(ctypes.byref(b), 0, ctypes.byref(cfg), *args) == _lib.RX_EINVAL


def test_schedule_config_is_validated_and_the_library_reads_no_environment():
    """ABI v17: the launch-schedule choices are rx_config fields
    with validated ranges -- out-of-range values fail rx_create with RX_EINVAL and
    a message naming the field, before any HIP call -- and the production library
    reads no environment variable at all (getenv is not among its imports), so a
    stray RX_* variable cannot change the product path."""
    import subprocess
    from rx import _build, _lib
    L = _lib.load()
    h = _lib._P()
    base = [16, 1, 11, 3000, 0, 0, 0, 1.0471975511965976, 8.0, 8, 16, 2, 8]
    bad = {"split": 2, "wide_n": -2, "dyn_lpe": 3, "ray_lpr": 8, "reward_lpe": 64, "argmin_window": 33,
           "seg_filter": 5, "box_quadrants": -3, "ray_dispatch": 4, "ray_tail": 17, "ray_tail_lpr": 3,
           "task_sort": 17, "lane_tracks": 2}
    for k, v in bad.items():
        sched = [v if f == k else 0 for f in _lib.SCHED_FIELDS]
        assert L.rx_create(_lib.RxConfig(*base, *sched), h) == _lib.RX_EINVAL, k
        assert k.encode() in L.rx_last_error(), (k, L.rx_last_error())
    # ABI v23: the dropped kin_sort slot is reserved0 and must be 0
    assert L.rx_create(_lib.RxConfig(*base, *[0] * len(_lib.SCHED_FIELDS), 1), h) == _lib.RX_EINVAL
    assert b"reserved0" in L.rx_last_error()
    two = list(base)
    two[1] = 2
    assert L.rx_create(_lib.RxConfig(*two, *[2 if f == "dyn_lpe" else 0 for f in _lib.SCHED_FIELDS]), h) \
        == _lib.RX_EINVAL
    assert L.rx_create(_lib.RxConfig(*two, *[4 if f == "reward_lpe" else 0 for f in _lib.SCHED_FIELDS]), h) \
        == _lib.RX_EINVAL  # two cars: reward_lpe 1 or 2 (a lane per car)
    # every in-range value passes validation (on a CPU-only host rx_create then fails at the device query)
    import torch
    if not torch.cuda.is_available():
        for k, vals in {"split": (-1, 1), "wide_n": (-1, 5), "dyn_lpe": (1, 2, 4, 64), "ray_lpr": (1, 2, 4),
                        "reward_lpe": (1, 2, 4), "argmin_window": (-1, 1, 32), "seg_filter": (-1, 1),
                        "box_quadrants": (-1, 1), "ray_dispatch": (-1, 1, 2, 3), "ray_tail": (-1, 1, 16),
                        "ray_tail_lpr": (2, 4), "task_sort": (1, 2, 16), "lane_tracks": (-1, 1)}.items():
            for v in vals:
                sched = [v if f == k else 0 for f in _lib.SCHED_FIELDS]
                assert L.rx_create(_lib.RxConfig(*base, *sched), h) != _lib.RX_EINVAL, (k, v)
    und = subprocess.run(["nm", "-D", "--undefined-only", _build.LIB], capture_output=True, text=True, check=True)
    syms = {ln.split()[-1].split("@")[0] for ln in und.stdout.splitlines() if ln.strip()}
    assert "getenv" not in syms and "secure_getenv" not in syms, "librx.so must not read the environment"
    strings = open(_build.LIB, "rb").read()
    for knob in (b"RX_SEG_FILTER", b"RX_SPLIT", b"RX_RAY_LPR", b"RX_REWARD_LPE", b"RX_DYN1_LPE", b"RX_WIDE_N",
                 b"RX_ARGMIN_WINDOW", b"RX_BOX_QUAD", b"RX_KIN_WPB", b"RX_RAYS_WPB", b"RX_RAYS_LDS"):
        assert knob not in strings, knob


def test_default_sort_interval():
    """rx.vector_env.default_sort_interval: re-sort every 8 dynamics launches for
    single-agent envs above 32,768, every 16 elsewhere (profiles/r04/probe_sort_interval.txt)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
    from rx.vector_env import default_sort_interval
    assert default_sort_interval(65536, 1) == 8
    assert default_sort_interval(32768, 1) == 16
    assert default_sort_interval(4096, 1) == 16
    assert default_sort_interval(65536, 2) == 16
