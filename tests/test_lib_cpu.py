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
