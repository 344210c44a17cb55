"""Build librx variants (extra -D defines) into build/variants/<name>.so for
bring-up A/Bs on the GPU box (loaded with RX_LIB_PATH)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
from rx import _build  # noqa: E402

VARIANTS = {}
for arg in sys.argv[1:]:
    name, _, defs = arg.partition("=")
    VARIANTS[name] = [d for d in defs.split(",") if d]
os.makedirs(os.path.join(ROOT, "build", "variants"), exist_ok=True)
for name, defs in VARIANTS.items():
    out = os.path.join(ROOT, "build", "variants", name + ".so")
    _build.build(out=out, defines=defs, verbose=False)
    print(name, defs, out, flush=True)
