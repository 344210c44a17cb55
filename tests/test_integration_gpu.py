"""the ctypes binding a reference maintainer would paste in
(environment/rx_binding.py) is executed verbatim from the document and stepped
beside rx.vector_env.RacingVectorEnv: observations, rewards and done flags must
be identical bit for bit (the binding replaces gym.vector.SyncVectorEnv at
agent/ppo.py:70; its reference RacingEnv objects are stood in by rx.envs
RacingEnv specs, which expose the same .track / .num_sensors members)."""
import os
import random
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _binding_source():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 2. Bind the C ABI directly"):doc.index("## 3.")]
    blocks = re.findall(r"```python\n(.*?)```", sec, re.S)
    assert len(blocks) == 1, "INTEGRATION.md §2 must hold exactly one python block"
    return blocks[0].replace("<repo>", ROOT)


def test_binding_compiles_without_device():
    compile(_binding_source(), "INTEGRATION.md#2", "exec")


@pytest.mark.gpu
def test_integration_binding_matches_vector_env():
    import rx  # noqa: F401  (sys.path: rx/lib/librx.so must exist)
    from rx.envs import RacingEnv
    from rx.track import gen_tracks
    from rx.vector_env import RacingVectorEnv
    ns = {}
    exec(compile(_binding_source(), "INTEGRATION.md#2", "exec"), ns)
    N = 512
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(num_tracks=N, seed=1)
    widths = [int(np.random.randint(6, 10)) for _ in range(N)]
    envs = [RacingEnv(num_sensors=11, track_pool=pool, track_id=i, track_width=widths[i]) for i in range(N)]
    reset, step, keep = ns["make_vector_env"](envs)
    v = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step")
    o_b = reset().clone()
    o_v = v.reset_device()
    assert torch.equal(o_b, o_v)
    g = torch.Generator(device="cuda").manual_seed(17)
    scale = torch.tensor([2.0, 1.0], device="cuda")
    shift = torch.tensor([-1.0, 0.0], device="cuda")
    ends = 0
    for t in range(400):
        a = torch.rand((N, 2), device="cuda", generator=g) * scale + shift
        ob, rb, db = step(a)
        ov, rv, dv = v.step_device(a)
        assert torch.equal(ob, ov) and torch.equal(rb, rv) and torch.equal(db, dv), t
        ends += int(db.sum())
    assert ends > 50
    # rx_steps through the binding (ABI v21): 24 open-loop steps from one call each side
    a = torch.rand((24, N, 2), device="cuda", generator=g) * scale + shift
    ob, rb, db = step.steps(a)
    ov, rv, dv = v.steps_device(a)
    assert torch.equal(ob, ov) and torch.equal(rb, rv) and torch.equal(db, dv)
    v.close()
    keep_h = keep[0]
    assert ns["L"].rx_destroy(keep_h) == 0
