"""Diagnostic: phase breakdown of the column-split finish (FIN_STAMP slots, s_memrealtime 100 MHz).

Uses a separate library built with -DMPPI_STAMPS (never the product .so):
  make -C husky-rover-mppi-isaacsim_amd/csrc OUT=$PWD/ab/stamps.so EXTRA=-DMPPI_STAMPS
Usage (GPU box): python profiles/ubench/stamps_fin.py ab/stamps.so [K] [H] [async 0|1]
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
    asyn = (sys.argv[4] != "0") if len(sys.argv) > 4 else True
    os.environ["MPPI_LIB_PATH"] = so
    from mppi_amd import _lib, scene
    lib = _lib.load_library(so)
    lib.mppi_debug_stamps.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    Z, hw, cm = scene.scene_c3()
    eng = _lib.Engine(_lib.make_params(K, H), 0)
    eng.set_async_tail(asyn)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, goal_x=65.0, goal_y=10.0))
    n = 64 * 16 * 6 + 1024 * 2 + 64 * 8 + 64 + 512
    rows = []
    wgs = []
    for i in range(12):
        eng.step("3d", i)
        if i >= 4:
            eng.outputs()
            buf = (C.c_uint64 * n)()
            assert lib.mppi_debug_stamps(buf, n) == 0
            allb = np.array(buf, dtype=np.float64)
            rows.append(allb[-576:-512])
            wgs.append(allb[-512:].reshape(128, 4))
    fs = np.median(np.array(rows), axis=0)
    us = lambda a, b: (fs[b] - fs[a]) / 100.0  # noqa: E731
    print(f"K={K} H={H} async={asyn}: finish phases (us, median of {len(rows)} steps, workgroup 0 / last)")
    print(f"  start -> scale table {us(0, 9):.2f}  -> columns reduced {us(9, 10):.2f}  -> counted (last) {us(10, 13):.2f}")
    print(f"  u_opt read {us(13, 1):.2f}  phase2 setup {us(1, 2):.2f}  filter {us(2, 12):.2f}  "
          f"v/w/sincos {us(12, 3):.2f}  outputs {us(3, 4):.2f}  signal {us(4, 5):.2f}")
    print(f"  total start -> signal {us(0, 5):.2f}")
    if fs[21] > fs[3]:
        print(f"  optimal rollout: chain {us(3, 21):.2f}  heights / wheels + output stores {us(21, 4):.2f}")
    cyc = lambda a, b: fs[32 + b] - fs[32 + a]  # noqa: E731
    print(f"  shader clock over start -> signal {cyc(0, 5) / us(0, 5):.0f} MHz; filter {cyc(2, 12):.0f} cycles "
          f"({cyc(2, 12) / us(2, 12):.0f} MHz), register levels {cyc(11, 15):.0f} cycles")
    w0 = np.array(wgs)
    wa = np.median(w0[:, :16, 3] - np.array(rows)[:, 0][:, None], axis=0) / 100.0
    print("  workgroup 0, each wave at the minima barrier (us from start): " + " ".join(f"{x:.2f}" for x in wa))
    if fs[19] > 0:
        print(f"  start -> m loads issued {us(0, 18):.2f}  -> m loads back (wave 0) {us(18, 19):.2f}  "
              f"-> dependent reload {us(19, 20):.2f}")
    if fs[16] > 0:
        print(f"  scale table: minima loaded {us(0, 16):.2f}  min tree {us(16, 17):.2f}  pair scales {us(17, 9):.2f}")
    if fs[11] > 0:
        print(f"  columns: leaf loads done {us(9, 11):.2f}  register levels {us(11, 15):.2f}  "
              f"shuffle/LDS levels {us(15, 10):.2f}")
    if fs[7] > 0:
        print(f"  filter: first 16 steps {us(2, 7):.2f}  next 48 {us(7, 8):.2f}  to loop end {us(8, 14):.2f}  "
              f"tail steps {us(14, 12):.2f}")


if __name__ == "__main__":
    main()
