"""Build librx.so (HIP kernels + C ABI) for gfx950 with hipcc, in-tree.

    python -m rx._build            (from self-play-racing_amd/)

Output: self-play-racing_amd/rx/lib/librx.so (git-ignored; travels to the GPU
box with the snapshot).  hipcc cross-compiles here without a GPU.
"""
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                    # self-play-racing_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "librx.so")
SOURCES = ["rx_kernels.hip", "rx_sort.hip", "rx_optim.hip", "rx_ppo.hip", "rx_api.cpp"]
HEADERS = ["rx_internal.h", "rx_math.h", "rx_sincos_table.h", "rx_policy.h", "rx_policy_mfma.h"]

ARCH = os.environ.get("RX_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off: no implicit FMA anywhere (bit-exact with the reference's
# unfused numpy arithmetic); explicit FMAs only via rx_math.h.
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", f"--offload-arch={ARCH}",
         "-Wall", "-Wno-unused-function", "-I" + CSRC, "-I" + INCLUDE]


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm not installed?)")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, "rx.h"), __file__]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, out=None, defines=()):
    """Compile librx.so (out: another .so path, with extra -D defines: profiling variants)."""
    lib = out or LIB
    if out is None and not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    objs = []
    cc = hipcc()
    for src in SOURCES:
        obj = os.path.join(LIBDIR, os.path.splitext(src)[0] + ".o")
        if out is not None:
            obj = os.path.splitext(out)[0] + "_" + os.path.splitext(src)[0] + ".o"
        cmd = [cc] + FLAGS + [f"-D{d}" for d in defines] + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        objs.append(obj)
    tmp = lib + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
