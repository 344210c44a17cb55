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
    assert L.rx_adam_workspace_floats(ctypes.byref(cfg)) == 33 * 2  # ceil(2050 / 64) norm blocks x 2 tensors
    # fused minibatch update (ABI v13): argument checks before any launch
    assert L.rx_ppo_update_workspace_floats(15, ctypes.byref(cfg)) > 0
    assert L.rx_ppo_update_workspace_floats(7, ctypes.byref(cfg)) == 0
    b.obs_dim = 15
    args = [None] * 12
    assert L.rx_ppo_minibatch_update(ctypes.byref(b), 0, ctypes.byref(cfg), *args) == _lib.RX_EINVAL
