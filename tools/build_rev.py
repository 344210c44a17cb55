"""Build librx.so from another git revision's sources, for same-session A/B runs.

    python tools/build_rev.py REV NAME [--only a.hip,b.h] [-DFLAG=V ...]  -> self-play-racing_amd/rx/lib/librx_NAME.so
    (REV "." = the working tree; extra arguments are added to the hipcc flags; --only takes just
    those csrc files from REV and the rest from the working tree, e.g. old kernels behind the
    current ABI)
    RX_LIB_PATH=.../librx_NAME.so python bench.py ...   (on the GPU box)

Only the C/HIP sources and headers are taken from REV; the Python side must
speak the same ABI (rx_abi_version is checked at load).
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
from rx import _build  # noqa: E402


def main():
    rev, name = sys.argv[1], sys.argv[2]
    extra = sys.argv[3:]
    only = None
    if "--only" in extra:
        i = extra.index("--only")
        only = set(extra[i + 1].split(","))
        extra = extra[:i] + extra[i + 2:]
    tmp = tempfile.mkdtemp(prefix="rxrev_")
    csrc = os.path.join(tmp, "csrc")
    inc = os.path.join(tmp, "include")
    os.makedirs(csrc)
    os.makedirs(inc)
    def read(path):
        if rev == "." or (only is not None and os.path.basename(path) not in only):
            return open(os.path.join(ROOT, path), "rb").read()
        return subprocess.check_output(["git", "-C", ROOT, "show", f"{rev}:{path}"])
    for f in _build.SOURCES + _build.HEADERS:
        open(os.path.join(csrc, f), "wb").write(read(f"self-play-racing_amd/csrc/{f}"))
    open(os.path.join(inc, "rx.h"), "wb").write(read("include/rx.h"))
    out = os.path.join(_build.LIBDIR, f"librx_{name}.so")
    flags = [x for x in _build.FLAGS if not x.startswith("-I")] + ["-I" + csrc, "-I" + inc] + extra
    objs = []
    for src in _build.SOURCES:
        obj = os.path.join(tmp, os.path.splitext(src)[0] + ".o")
        subprocess.check_call([_build.hipcc()] + flags + ["-c", os.path.join(csrc, src), "-o", obj])
        objs.append(obj)
    subprocess.check_call([_build.hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out] + objs)
    print(out)


if __name__ == "__main__":
    main()
