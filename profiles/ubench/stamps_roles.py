"""Diagnostic: per-role work / wait cycles per step of the role-split rollout kernel.

Uses a separate library built with -DMPPI_STAMPS (never the product .so):
  make -C husky-rover-mppi-isaacsim_amd/csrc OUT=$PWD/ab/stamps.so EXTRA=-DMPPI_STAMPS
Usage (GPU box): python profiles/ubench/stamps_roles.py ab/stamps.so [K] [H]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]


def main():
    so = os.path.abspath(sys.argv[1])
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    os.environ["MPPI_LIB_PATH"] = so
    from mppi_amd import _lib, scene
    lib = _lib.load_library(so)
    lib.mppi_debug_stamps.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    Z, hw, cm = scene.scene_c3()
    eng = _lib.Engine(_lib.make_params(K, H), 0)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, goal_x=65.0, goal_y=10.0))
    for i in range(5):
        eng.step("3d", i)
    n = 64 * 16 * 3
    buf = (C.c_uint64 * n)()
    assert lib.mppi_debug_stamps(buf, n) == 0
    v = np.array(buf, dtype=np.float64)
    nb = min(64, (K + 255) // 256)
    ww = v[:64 * 16 * 2].reshape(64, 16, 2)[:nb] / H
    cnt = v[64 * 16 * 2:64 * 16 * 3].reshape(64, 16)[:nb] / H
    names = ["chain", "prod", "wheel", "cost"]
    print(f"K={K} H={H}: cycles per step (mean over {nb} workgroups x 4 groups)")
    for r, nm in enumerate(names):
        w = ww[:, 4 * r:4 * r + 4]
        print(f"  {nm:6s} work {w[..., 0].mean():8.1f}  wait {w[..., 1].mean():8.1f}  "
              f"LDS waits/step {cnt[:, 4 * r:4 * r + 4].mean():5.2f}")
    # leaf_records stamps of thread 0 (the chain wave of group 0; s_memtime cycles):
    # 0 entry, 1 after the weights (its first barrier waits for every role's last step),
    # 4 after the rows (loads + float64 line sums), 5 after the record tree and stores
    n2 = 64 * 16 * 6 + 1024 * 2 + 64 * 8
    b2 = (C.c_uint64 * n2)()
    assert lib.mppi_debug_stamps(b2, n2) == 0
    lf = np.array(b2, dtype=np.float64)[64 * 16 * 6 + 1024 * 2:].reshape(64, 8)[:nb]
    if lf[:, 5].max() > 0:
        print(f"  leaf (cycles, mean over {nb} workgroups): barrier+weights {np.mean(lf[:, 1] - lf[:, 0]):7.0f}  "
              f"rows {np.mean(lf[:, 4] - lf[:, 1]):7.0f}  record {np.mean(lf[:, 5] - lf[:, 4]):7.0f}  "
              f"total {np.mean(lf[:, 5] - lf[:, 0]):7.0f}")


if __name__ == "__main__":
    main()
