"""Shared test helpers: scenes, oracle/engine builders, comparisons."""
from __future__ import annotations

import functools

import numpy as np

from mppi_amd import scene
from oracle import mppi_ref as R

START = (-60.0, -5.0)
GOAL = (65.0, 10.0)


@functools.lru_cache(maxsize=1)
def c3_scene():
    """C1-C4 scene (1500^2 DEM @0.1 m, 750^2 costmap @0.2 m), generated from the reference recipes."""
    Z, hw, cm = scene.scene_c3()
    return Z, hw, cm


def oracle_scene(Z, hw, cm):
    return R.Scene(Z, hw, cm)


def oracle_state(x=START[0], y=START[1], heading=(1.0, 0.0, 0.0), wl=0.0, wr=0.0, goal=GOAL,
                 s1=0.25, s2=0.25):
    return R.State(x=x, y=y, heading=np.asarray(heading, float), left_wheel_speed=wl,
                   right_wheel_speed=wr, goal_x=goal[0], goal_y=goal[1], std_dev_u1=s1, std_dev_u2=s2)


def engine_for(K, H, Z, hw, cm, st: R.State, seed=42, k_offset=0, device=0, **kw):
    from mppi_amd import _lib
    eng = _lib.Engine(_lib.make_params(K, H, k_offset=k_offset, seed=seed, **kw), device)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(state_for(st))
    return eng


def state_for(st: R.State):
    from mppi_amd import _lib
    return _lib.make_state(st.x, st.y, st.heading, st.left_wheel_speed, st.right_wheel_speed,
                           st.goal_x, st.goal_y, st.std_dev_u1, st.std_dev_u2)


def rel_err(a, b, floor=1e-3):
    """max |a-b| / max(|b|, floor) — the north-star tolerance metric on the emitted controls."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor)))


def mismatch_report(name, got, want, n=5):
    got = np.asarray(got)
    want = np.asarray(want)
    bad = np.nonzero(got.reshape(-1) != want.reshape(-1))[0]
    if bad.size == 0:
        return f"{name}: identical"
    idx = bad[:n]
    return (f"{name}: {bad.size}/{got.size} differ; first idx {idx.tolist()} got "
            f"{got.reshape(-1)[idx].tolist()} want {want.reshape(-1)[idx].tolist()}")
