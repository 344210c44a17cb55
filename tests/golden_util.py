"""Loaders for the committed golden vectors (tests/golden/*.npz).

The vectors were produced from the reference by tests/golden/gen_golden.py (in
the build container); here they are data only -- no reference code is needed or
read at test time, so these tests also run on the GPU box.
"""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def unpack(cat, off, k):
    return cat[off[k]:off[k + 1]]


class Golden:
    def __init__(self):
        self.geo = load("geometry.npz")
        g = self.geo
        self.n_tracks = len(g["width"])
        self.tracks = []
        for k in range(self.n_tracks):
            self.tracks.append(dict(
                cp=unpack(g["cp"], g["cp_off"], k),
                wp=unpack(g["wp"], g["wp_off"], k),
                nrm=unpack(g["nrm"], g["nrm_off"], k),
                starts=unpack(g["starts"], g["starts_off"], k),
                v2=unpack(g["v2"], g["v2_off"], k),
                start=g["start"][k], width=float(g["width"][k]), maxd=float(g["maxd"][k]),
                label=str(g["labels"][k])))
        self._cache = {}

    def table(self):
        from oracle.orc import TrackTable
        if "table" not in self._cache:
            self._cache["table"] = TrackTable(self.tracks)
        return self._cache["table"]

    def __getitem__(self, name):
        if name not in self._cache:
            self._cache[name] = load(name + ".npz")
        return self._cache[name]


def single_state_from(step, idx=None):
    """Build an SoA single-env state (oracle/device layout) from step_single.npz inputs."""
    sl = slice(None) if idx is None else idx
    n = len(step["x"][sl])
    st = {}
    for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering"):
        st[k] = np.ascontiguousarray(step[k][sl], dtype=np.float64)
    st["steps"] = np.ascontiguousarray(step["steps"][sl], dtype=np.int32)
    st["track"] = np.ascontiguousarray(step["track"][sl], dtype=np.int32)
    cp = step["cp"][sl]
    fl = (step["crashed"][sl].astype(np.uint8) * 1 + step["finished"][sl].astype(np.uint8) * 2
          + cp[:, 0] * 4 + cp[:, 1] * 8 + cp[:, 2] * 16)
    st["flags"] = np.ascontiguousarray(fl, dtype=np.uint8)
    assert len(st["x"]) == n
    return st


def multi_state_from(step):
    n = len(step["steps"])
    st = {}
    for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering"):
        st[k] = np.ascontiguousarray(step[k], dtype=np.float64)
    st["finished_step"] = np.ascontiguousarray(step["finished_step"], dtype=np.int32)
    cp = step["cp"]
    fl = (step["crashed"].astype(np.uint8) + step["finished"].astype(np.uint8) * 2 + cp[:, :, 0] * 4
          + cp[:, :, 1] * 8 + cp[:, :, 2] * 16 + step["has_crashed"].astype(np.uint8) * 32)
    st["flags"] = np.ascontiguousarray(fl, dtype=np.uint8)
    st["steps"] = np.ascontiguousarray(step["steps"], dtype=np.int32)
    st["track"] = np.ascontiguousarray(step["track"], dtype=np.int32)
    assert st["x"].shape == (n, 2)
    return st
