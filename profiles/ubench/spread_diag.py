"""Diagnostic (not part of the product): which rollout workgroups end late.  C3, separate launches
in timing mode 2 (each rollout isolated from side-stream work) and on the resident server; per
workgroup the time from the first start to its record (chain-clock stamps of the last rollout),
grouped by blockIdx % 8 (the XCD group) and the slowest workgroups listed."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd"))
from mppi_amd import _lib, scene  # noqa: E402
import ctypes as C  # noqa: E402

Z, hw, cm = scene.scene_c3()
for mode in ("timing2", "server", "separate"):
    eng = _lib.Engine(_lib.make_params(65536, 100), 0)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
    eng.set_async_tail(True)
    if mode == "timing2":
        eng.set_timing(2)
    if mode == "separate":
        eng.set_option("resident", 0)
    rows = []
    for rep in range(6):
        for i in range(30):
            eng.step("3d", rep * 100 + i, copy=False)
        v = (C.c_double * 300)()
        eng._c(eng.lib.mppi_get_chain_clock(eng.ctx, v, 300), "mppi_get_chain_clock")
        rec = np.array([v[10 + b] for b in range(256)])
        start_spread = v[7]
        rows.append(rec)
        order = np.argsort(rec)[::-1][:6]
        print(f"{mode} rep {rep}: p50 {np.median(rec):.1f} max {rec.max():.1f} start spread {start_spread:.1f}; "
              f"by blockIdx%8 max: " + " ".join(f"{rec[g::8].max():.1f}" for g in range(8)) +
              "; slowest " + " ".join(f"{b}({rec[b]:.1f})" for b in order))
    r = np.array(rows)
    late = (r > np.median(r, axis=1, keepdims=True) + 3.0).sum(0)
    print(f"{mode}: workgroups late (> p50 + 3 us) in >= 3 of 6 reps: {list(np.nonzero(late >= 3)[0])}")
    eng.close()
