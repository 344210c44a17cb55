"""Probe: does a hipcc-built C-ABI .so share torch's HIP runtime, and how do
device f64 sin/cos/div/sqrt/fmod and f32 div compare with host glibc/numpy?"""
import ctypes, os, sys, time
import numpy as np
import torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libm_probe.so"))
lib.run.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
print(torch.cuda.get_device_name(0), torch.version.hip)
n = 1 << 20
rng = np.random.default_rng(0)
xs = rng.uniform(-2.0, 8.5, n)
ys = rng.uniform(0.1, 50.0, n)
a = torch.from_numpy(xs).to(dev); c = torch.from_numpy(ys).to(dev)
b = torch.empty_like(a)
s = torch.cuda.current_stream().cuda_stream
def run(which, a_, c_, b_):
    r = lib.run(which.encode(), ctypes.c_void_p(a_.data_ptr()), ctypes.c_void_p(c_.data_ptr()), ctypes.c_void_p(b_.data_ptr()), a_.numel(), ctypes.c_void_p(s))
    torch.cuda.synchronize(); assert r == 0, r
    return b_.cpu().numpy()
out = run("sin", a, c, b); ref = np.sin(xs); print("sin mismatch vs glibc:", int((out != ref).sum()), "/", n, "maxulp", int(np.max(np.abs(out.view(np.int64) - ref.view(np.int64)))))
out = run("cos", a, c, b); ref = np.cos(xs); print("cos mismatch vs glibc:", int((out != ref).sum()), "/", n, "maxulp", int(np.max(np.abs(out.view(np.int64) - ref.view(np.int64)))))
out = run("div", a, c, b); ref = xs / ys; print("div mismatch:", int((out != ref).sum()))
a2 = torch.from_numpy(ys * 37.0).to(dev)
out = run("sqrt", a2, c, b); ref = np.sqrt(ys * 37.0); print("sqrt mismatch:", int((out != ref).sum()))
xm = rng.uniform(-10, 20, n); am = torch.from_numpy(xm).to(dev)
out = run("mod", am, c, b); ref = np.fmod(xm, 6.283185307179586); print("fmod mismatch:", int((out != ref).sum()))
xf = rng.uniform(0, 200, n).astype(np.float32); af = torch.from_numpy(xf).to(dev); bf = torch.empty_like(af)
out = run("fdiv", af, af, bf); ref = xf / np.float32(50.0); print("f32 div mismatch:", int((out != ref).sum()))
print("interop OK")
