"""Diagnostic: per-workgroup record times of the C3 rollout (mppi_get_chain_clock out[10 + b]),
pipelined (deferred tail) and synchronous steps.  Usage (GPU box): python profiles/ubench/wg_ends.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]


def main():
    from mppi_amd import _lib, scene
    Z, hw, cm = scene.scene_c3()
    eng = _lib.Engine(_lib.make_params(65536, 100), 0)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, goal_x=65.0, goal_y=10.0))
    for mode in ("pipelined", "sync", "pipelined"):
        eng.set_async_tail(mode == "pipelined")
        rows = []
        for i in range(60):
            eng.step("3d", i, copy=False)
            if i >= 40:
                v = (C.c_double * (10 + 256))()
                assert eng.lib.mppi_get_chain_clock(eng.ctx, v, 10 + 256) == 0
                rows.append(np.array(v[10:10 + 256]))
        a = np.array(rows)                      # [steps, 256] record times
        ends = np.sort(a, axis=1)
        print(f"{mode}: record time per workgroup, median over 20 steps (us): min {np.median(ends[:, 0]):.1f} "
              f"p10 {np.median(ends[:, 25]):.1f} p50 {np.median(ends[:, 128]):.1f} p90 {np.median(ends[:, 230]):.1f} "
              f"p99 {np.median(ends[:, 253]):.1f} max {np.median(ends[:, 255]):.1f}")
        slow = np.argsort(a.mean(axis=0))[-8:]
        print("   slowest workgroups (mean):", [(int(b), round(float(a[:, b].mean()), 1)) for b in slow])
    eng.close()


if __name__ == "__main__":
    main()
