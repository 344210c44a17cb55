"""Flat-buffer Adam for the PPO update (agent/ppo.py:83,204-207) on one HIP launch.

``FlatAdam(module, optimizer, max_grad_norm)`` moves every parameter of the
policy into ONE contiguous float32 buffer (``p.data`` becomes a view; the
Parameter objects, their names and the module's state_dict are unchanged) and
pre-assigns ``p.grad`` as views of one flat gradient buffer, which autograd
then accumulates into in place.  That gives:

* ``step(stop)``: clip_grad_norm_ + Adam in two launches (rx_adam_clip_step),
  with lr / step count / early-stop flag in device memory -> graph-capturable;
* one flat gradient tensor for the data-parallel all-reduce (rx.dist), with
  the minibatch KL in the slot after it (``bucket``: grad + KL in ONE
  all-reduce);
* the torch ``optimizer`` stays the source of truth for the API: its
  param_groups carry lr/betas/eps (the lr anneal writes there), and
  ``export_state()`` / ``import_state()`` move the moments and step count in
  and out of its ``state`` so ``optimizer.state_dict()`` checkpoints keep the
  reference format (agent/self_play_ppo.py:146-159).

No CPU path: the launch goes through librx and fails loudly without it.
"""
import ctypes

import torch

from . import _lib


class FlatParams:
    """A module's float32 parameters moved into ONE contiguous buffer (``p.data``
    become views; names, state_dict and load_state_dict are unchanged).  What
    rx_policy_act needs for a module that is never optimised (the frozen
    self-play opponent)."""

    def __init__(self, module):
        params = [p for p in module.parameters()]
        if not params or any(p.dtype != torch.float32 for p in params):
            raise ValueError("FlatParams expects float32 parameters")
        self.flat_param = torch.empty(sum(p.numel() for p in params), dtype=torch.float32, device=params[0].device)
        o = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                self.flat_param[o:o + k].copy_(p.reshape(-1))
                p.data = self.flat_param[o:o + k].view_as(p)
                o += k


class FlatAdam:
    def __init__(self, module, optimizer, max_grad_norm):
        self.module = module
        self.optimizer = optimizer
        self.max_grad_norm = float(max_grad_norm)
        self.params = [p for p in module.parameters()]
        if len(self.params) > _lib.ADAM_MAX_TENSORS:
            raise ValueError(f"{len(self.params)} parameter tensors > {_lib.ADAM_MAX_TENSORS}")
        dev = self.params[0].device
        if dev.type != "cuda":
            raise RuntimeError("FlatAdam needs the policy on a HIP device")
        sizes = [p.numel() for p in self.params]
        n = sum(sizes)
        self.numel = n
        self.flat_param = torch.empty(n, dtype=torch.float32, device=dev)
        # one all-reduce bucket: the flat gradient and, right after it, the
        # data-parallel update's KL slot (rx_ppo_minibatch_grad_shard)
        self.bucket = torch.zeros(n + 1, dtype=torch.float32, device=dev)
        self.flat_grad = self.bucket[:n]
        self.kl_slot = self.bucket[n:]
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step_t = torch.zeros((), dtype=torch.float32, device=dev)
        self.lr_t = torch.zeros((), dtype=torch.float64, device=dev)
        self.views = []
        o = 0
        with torch.no_grad():
            for p, k in zip(self.params, sizes):
                if p.dtype != torch.float32:
                    raise ValueError("FlatAdam expects float32 parameters")
                sl = slice(o, o + k)
                self.flat_param[sl].copy_(p.reshape(-1))
                p.data = self.flat_param[sl].view_as(p)
                p.grad = self.flat_grad[sl].view_as(p)
                self.views.append(sl)
                o += k
        g = optimizer.param_groups[0]
        if len(optimizer.param_groups) != 1 or g.get("weight_decay", 0) or g.get("amsgrad", False) \
                or g.get("maximize", False):
            raise ValueError("FlatAdam mirrors a single-group plain Adam (agent/ppo.py:83)")
        b1, b2 = g["betas"]
        offs = [0]
        for k in sizes:
            offs.append(offs[-1] + k)
        self.cfg = _lib.RxAdamConfig(len(sizes), (ctypes.c_int64 * 33)(*offs), float(b1), float(b2),
                                     float(g["eps"]), self.max_grad_norm)
        self.ws = torch.empty(_lib.load().rx_adam_workspace_floats(ctypes.byref(self.cfg)), dtype=torch.float32,
                              device=dev)
        if self.ws.numel() == 0:
            raise RuntimeError(_lib.load().rx_last_error().decode())
        self.import_state()

    def zero_grad(self):
        self.flat_grad.zero_()

    def sync_lr(self):
        """Copy optimizer.param_groups[0]['lr'] (set by the anneal) to the device scalar."""
        self.lr_t.fill_(float(self.optimizer.param_groups[0]["lr"]))

    def step(self, stop=None, stream=None):
        L = _lib.load()
        if stop is not None and (stop.dtype != torch.bool or stop.numel() != 1 or not stop.is_cuda):
            raise ValueError("stop must be a 1-element device bool tensor")
        _lib.check(L.rx_adam_clip_step(ctypes.byref(self.cfg), _lib.ptr(self.flat_param), _lib.ptr(self.flat_grad),
                                       _lib.ptr(self.exp_avg), _lib.ptr(self.exp_avg_sq), _lib.ptr(self.step_t),
                                       _lib.ptr(self.lr_t), _lib.ptr(stop) if stop is not None else None,
                                       _lib.ptr(self.ws), _lib.stream_ptr(stream)), "rx_adam_clip_step")

    # ------------------------------------------------------------ torch.optim interop
    def export_state(self):
        """Write step / exp_avg / exp_avg_sq into optimizer.state (reference format)."""
        step = float(self.step_t.item())
        if step == 0.0:
            return
        for p, sl in zip(self.params, self.views):
            self.optimizer.state[p] = {"step": torch.tensor(step, dtype=torch.float32),
                                       "exp_avg": self.exp_avg[sl].view_as(p).clone(),
                                       "exp_avg_sq": self.exp_avg_sq[sl].view_as(p).clone()}

    def import_state(self):
        """Load optimizer.state (e.g. after optimizer.load_state_dict) into the flat buffers."""
        st = [self.optimizer.state.get(p) for p in self.params]
        if not any(st):
            return
        with torch.no_grad():
            for p, sl, s in zip(self.params, self.views, st):
                if s:
                    self.exp_avg[sl].copy_(s["exp_avg"].reshape(-1))
                    self.exp_avg_sq[sl].copy_(s["exp_avg_sq"].reshape(-1))
            steps = {float(s["step"]) for s in st if s}
            if len(steps) != 1:
                raise ValueError(f"inconsistent Adam step counts {steps}")
            self.step_t.fill_(steps.pop())

    def rebind(self):
        """Re-point p.data / p.grad at the flat buffers (after something replaced them)."""
        with torch.no_grad():
            for p, sl in zip(self.params, self.views):
                v = self.flat_param[sl].view_as(p)
                if p.data_ptr() != v.data_ptr():
                    v.copy_(p.data)
                    p.data = v
                p.grad = self.flat_grad[sl].view_as(p)
