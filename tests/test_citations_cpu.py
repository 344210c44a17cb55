"""Every `<reference file>.py:<line>[-<line>]` citation in the boundary header
and the design notes points inside the cited reference file (skipped where the
reference tree is absent, e.g. on the GPU box)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
DOCS = ("include/rx.h", "DESIGN.md", "INTEGRATION.md")


def _ref_files():
    out = {}
    for d, _, fs in os.walk(REF):
        if "/." in d:
            continue
        for f in fs:
            if f.endswith(".py"):
                p = os.path.join(d, f)
                out.setdefault(f, []).append(p)
                out[os.path.relpath(p, REF)] = [p]
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
@pytest.mark.parametrize("doc", DOCS)
def test_citations_point_inside_the_reference(doc):
    files = _ref_files()
    text = open(os.path.join(ROOT, doc)).read()
    bad = []
    for m in re.finditer(r"([\w/]+\.py):(\d+(?:-\d+)?(?:,\d+(?:-\d+)?)*)", text):
        name, spans = m.group(1), m.group(2)
        cands = files.get(name) if "/" in name else files.get(name)
        if not cands:
            continue  # not a reference file (this repo's own modules)
        n = max(sum(1 for _ in open(p, errors="replace")) for p in cands)
        for span in spans.split(","):
            hi = int(span.split("-")[-1])
            if hi > n:
                bad.append(f"{m.group(0)} (file has {n} lines)")
    assert not bad, bad
