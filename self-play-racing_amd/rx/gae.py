"""GAE on the device -- PPO.compute_advantages (agent/ppo.py:134-154) as one HIP
kernel instead of T x ~6 tiny torch launches."""
import torch

from . import _lib


def compute_gae(rewards, dones, values, next_value, next_done, gamma, gae_lambda, scan=False, out=None, stream=None):
    """rewards/dones/values: float32 [T, N] device tensors; next_value [N];
    next_done [N] (bool or float).  Returns (advantages, returns) [T, N].

    scan=False: lane-per-env recurrence, bit-exact with the reference.
    scan=True : wavefront-parallel affine scan over T (few envs, long horizon);
                equal to within ~1e-6 relative."""
    L = _lib.load()
    T, N = rewards.shape
    for t in (rewards, dones, values):
        if t.shape != (T, N) or t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError("rewards/dones/values must be float32 [T, N] device tensors")
    nv = next_value.reshape(N).to(torch.float32).contiguous()
    nd = next_done.reshape(N).to(torch.float32).contiguous()
    r, d, v = rewards.contiguous(), dones.contiguous(), values.contiguous()
    if out is None:
        adv = torch.empty_like(r)
        ret = torch.empty_like(r)
    else:
        adv, ret = out
    fn = L.rx_gae_scan if scan else L.rx_gae
    _lib.check(fn(T, N, _lib.ptr(r), _lib.ptr(v), _lib.ptr(d), _lib.ptr(nv), _lib.ptr(nd), float(gamma),
                  float(gae_lambda), _lib.ptr(adv), _lib.ptr(ret), _lib.stream_ptr(stream)), "rx_gae")
    return adv, ret
