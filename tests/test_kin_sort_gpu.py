"""k_kin1p (rx_config.kin_sort, ABI v22; DESIGN.md §3 "Ray-task ranking"):
the sorting KIN launch with the ray-task ranking spread over a 4-wave workgroup
against k_kin1, whose single kinematics wave ranks all of its block's tasks.

The task list is scheduling only: k_step2's ray waves read it, no result depends
on its order.  What both kernels must write is the same counting sort: at EVERY
position of the device task list (rx_ray_tasks) a task of the same direction
sector -- recomputed here on the host from the stepped angles with the kernels'
float32 sector arithmetic -- and inside each run of one sector the same tasks.
The order inside a run is the order in which the LDS returns the ds_add_rtn
ranks of conflicting lanes, a hardware artefact that differs between the two
kernels (measured: lane 55's task after lanes 62 and 63 in k_kin1p).  Every
step's outputs and the whole f64 state must be equal bit for bit.
"""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _seed1_pool(n):
    from rx.track import gen_tracks
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(num_tracks=n, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(n)]
    return pool, widths


def _sectors(v, tasks):
    """The direction sector of each task id p*R + r (k_kin1 / k_kin1p: the stepped
    angle plus the ray's offset, to float32, 64 sectors per turn)."""
    R = v.n_sensors
    perm, _, _ = v.env_order()
    ang = v.get_state()["angle"]
    p, r = tasks // R, tasks % R
    th = (ang[perm[p]] + v.sensor_angles[r]).astype(np.float32)
    inv = np.float32(64.0) * np.float32(0.15915494309189535)
    return np.floor(th * inv).astype(np.int64) & 63


@pytest.mark.parametrize("N,sched", [(65536, {}), (4096, dict(ray_lpr=1, reward_lpe=1, task_sort=1)),
                                     (3001, dict(task_sort=1))])
def test_kin_sort_same_counting_sort_as_k_kin1(N, sched):
    from rx.vector_env import RacingVectorEnv
    pool, widths = _seed1_pool(N)
    # no spatial re-sort: the env order (and so every task id) stays fixed between the two
    kw = dict(device="cuda", autoreset="next_step", sort_interval=0)
    on = RacingVectorEnv(pool, widths, sched={**sched, "kin_sort": 1}, **kw)
    off = RacingVectorEnv(pool, widths, sched={**sched, "kin_sort": -1}, **kw)
    assert on.schedule()["kin_sort"] == 1 and off.schedule()["kin_sort"] == 0
    assert np.array_equal(on.env_order()[0], off.env_order()[0])
    assert torch.equal(on.reset_device(), off.reset_device())
    g = torch.Generator(device="cuda").manual_seed(N)
    for t in range(24):
        a = torch.rand((N, 2), device="cuda", generator=g)
        a[:, 0].mul_(2.0).sub_(1.0)
        outs = [v.step_device(a) for v in (on, off)]
        for x, y in zip(*outs):
            assert torch.equal(x, y), t
        if t % 6 != 5:
            continue
        ta, tb = on.ray_tasks(), off.ray_tasks()
        assert len(ta) == N * on.n_sensors
        assert np.array_equal(np.sort(ta), np.arange(len(ta)))  # a permutation of the tasks
        assert not np.array_equal(ta, np.arange(len(ta)))  # and a sorted one
        sa, sb = _sectors(on, ta), _sectors(off, tb)
        assert np.array_equal(sa, sb), (t, int(np.argmax(sa != sb)))  # same sector at every position
        run = np.concatenate([[0], np.cumsum(sa[1:] != sa[:-1])])
        oa, ob = np.lexsort((ta, run)), np.lexsort((tb, run))
        assert np.array_equal(ta[oa], tb[ob]), t  # the same tasks inside every run
    sa, sb = on.get_state(), off.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    on.close()
    off.close()
