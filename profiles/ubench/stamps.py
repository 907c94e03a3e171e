"""Diagnostic: per-wave work / barrier-wait cycles of the warp-specialised rollout kernel.

Builds a separate library with -DMPPI_STAMPS (never the product .so), runs C3
steps and prints average cycles per phase for chain and side waves.
Usage (GPU box): python profiles/ubench/stamps.py [K]
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")
sys.path[:0] = [ROOT, PKG]
SO = os.environ.get("MPPI_STAMPS_SO") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmppi_hip_stamps.so")


def build():
    csrc = os.path.join(PKG, "csrc")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
           "-fPIC", "-shared", "-DMPPI_STAMPS", f"-I{ROOT}/include", f"-I{csrc}", "-x", "hip",
           *[os.path.join(csrc, f) for f in ("mppi_kernels.hip", "mppi_costmap.hip", "mppi_python25d.hip",
                                            "mppi_capi.cpp")], "-o", SO]
    subprocess.run(cmd, check=True)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    path = sys.argv[2] if len(sys.argv) > 2 else "pair"
    if not os.path.exists(SO):
        build()
    from mppi_amd import _lib, scene
    lib = _lib.load_library(SO)
    lib.mppi_debug_stamps.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    _lib._lib = lib  # Engine uses the stamps build
    Z, hw, cm = scene.scene_c3()
    H = 100
    eng = _lib.Engine(_lib.make_params(K, H), 0)
    eng.set_dem_path(path)
    eng.set_async_tail(True)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, goal_x=65.0, goal_y=10.0))
    for i in range(5):
        eng.step("3d", i, copy=False)
    n = 64 * 16 * 2 + 64 * 16 * 4 + 1024 * 2 + 64 * 8 + 16
    buf = (C.c_uint64 * n)()
    assert lib.mppi_debug_stamps(buf, n) == 0
    allv = np.array(buf, dtype=np.float64)
    nb_all = (K + 255) // 256
    se = allv[64 * 16 * 6: 64 * 16 * 6 + 2 * nb_all].reshape(nb_all, 2)
    t0 = se[:, 0].min()
    st, en = (se[:, 0] - t0) / 100.0, (se[:, 1] - t0) / 100.0
    print(f"  block start (us): min {st.min():.1f} median {np.median(st):.1f} max {st.max():.1f}; "
          f"end: min {en.min():.1f} median {np.median(en):.1f} max {en.max():.1f}")
    print("  start histogram (10 us bins):", np.histogram(st, bins=np.arange(0, st.max() + 10, 10))[0].tolist())
    # per-wave slots: (block * 8 + wave) * 2 and 2048 + (block * 8 + wave) * 4 (8 waves per block)
    a = allv[:64 * 8 * 2].reshape(64, 8, 2)
    b = allv[64 * 16 * 2: 64 * 16 * 2 + 64 * 8 * 4].reshape(64, 8, 4)[: min(64, (K + 255) // 256)]
    print(f"  loop+cost {b[..., 0].mean():10.0f} cyc   leaf records {b[..., 1].mean():8.0f} cyc   "
          f"total {b[..., 3].mean():10.0f} cyc = {b[..., 2].mean() / 100:8.1f} us wall "
          f"-> clock {b[..., 3].mean() / (b[..., 2].mean() * 10):.2f} GHz")
    nb = min(64, (K + 255) // 256)
    a = a[:nb, :8]
    phases = H + 2
    chain = a[:, :4].reshape(-1, 2) / phases
    side = a[:, 4:].reshape(-1, 2) / phases
    lf = allv[64 * 16 * 6 + 1024 * 2: 64 * 16 * 6 + 1024 * 2 + 64 * 8].reshape(64, 8)[:nb]
    fs = allv[64 * 16 * 6 + 1024 * 2 + 64 * 8:][:16]
    if lf[:, 4].max() > 0:  # leaf_records stamps (thread 0 of each block, s_memtime cycles)
        print(f"  leaf records (cyc): weights {np.mean(lf[:, 1] - lf[:, 0]):8.0f}  "
              f"rows {np.mean(lf[:, 4] - lf[:, 1]):8.0f}  (block 0 total {lf[0, 4] - lf[0, 0]:.0f})")
    us = lambda a, b: (fs[b] - fs[a]) / 100.0  # s_memrealtime: 100 MHz, comparable across CUs
    if fs[13] > 0:
        print(f"  finish level1 (us): scales {us(0, 9):.1f}  apply+store {us(9, 10):.1f}  count {us(10, 13):.1f}; "
              f"last group: scales {us(13, 6):.1f}  apply {us(6, 1):.1f}; phase2 prologue {us(1, 2):.1f}")
        print(f"  previous finish signal -> this rollout's block 0 start: {us(14, 15):.1f} us")
        print(f"  finish kernel (us): level1 {us(0, 13):.1f}  rest of tree {us(13, 1):.1f}  "
              f"filter {us(2, 12):.1f}  v/w/sincos {us(12, 3):.1f}  outputs {us(3, 4):.1f}  signal {us(4, 5):.1f}")
    else:
        print(f"  finish kernel (us): tree {us(0, 1):.1f}  filter {us(2, 12):.1f}  v/w/sincos {us(12, 3):.1f}  "
              f"outputs {us(3, 4):.1f}  signal {us(4, 5):.1f}")
    print(f"K={K} kernel={path}: cycles per step (mean over {nb} blocks)")
    print(f"  chain waves: work {chain[:, 0].mean():8.1f}  wait {chain[:, 1].mean():8.1f}")
    print(f"  side  waves: work {side[:, 0].mean():8.1f}  wait {side[:, 1].mean():8.1f}")


if __name__ == "__main__":
    main()
