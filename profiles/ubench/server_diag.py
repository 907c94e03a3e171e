"""Diagnostic (not part of the product): host-side timing of the resident step server's calls.
Per step: mppi_step wall time, mppi_get_outputs wall time (waits for the deferred tail), and the
server launch count, for the deferred-tail and the synchronous modes, C3 (K 65536, H 100)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd"))
from mppi_amd import _lib, scene  # noqa: E402

Z, hw, cm = scene.scene_c3()
H = int(sys.argv[1]) if len(sys.argv) > 1 else 100
for async_tail in (True, False):
    eng = _lib.Engine(_lib.make_params(65536, H), 0)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
    eng.set_async_tail(async_tail)
    rows = []
    for i in range(12):
        t0 = time.perf_counter()
        eng.step("3d", i, copy=False)
        t1 = time.perf_counter()
        if i % 3 == 2:
            eng.outputs()
        t2 = time.perf_counter()
        rows.append((i, (t1 - t0) * 1e6, (t2 - t1) * 1e6, eng.launch_info()["server_launches"]))
    t0 = time.perf_counter()
    n = 200
    for i in range(12, 12 + n):
        eng.step("3d", i, copy=False)
    eng.outputs()
    dt = (time.perf_counter() - t0) / n * 1e6
    info = eng.launch_info()
    import ctypes as C
    import numpy as np
    v = (C.c_double * 400)()
    eng._c(eng.lib.mppi_get_chain_clock(eng.ctx, v, 400), "mppi_get_chain_clock")
    print(f"  last step: chain {v[1]:.0f} cyc/step {v[2]:.1f} us, wg0 leaf {v[6]:.1f} us, wg start spread {v[7]:.1f}, "
          f"end spread {v[8]:.1f}, span {v[9]:.1f} us")
    rec = np.array([v[10 + b] for b in range(256)])
    print("  per-workgroup record time from the first start (us): min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f; "
          "workgroup 0 %.1f (rank %d)" % (rec.min(), *np.percentile(rec, [10, 50, 90]), rec.max(), rec[0],
                                           int((rec < rec[0]).sum())))
    st = np.array([[v[266 + 8 * r + k] for k in range(8)] for r in range(8)])
    print("  server timeline, last 8 steps (us): [cmd seen, rollout = last ticket - cmd, finish = done - last ticket, "
          "noise end - done, next cmd - done, head poll start - done, last workgroup end - done, tail: gate - done, run]")
    for r in range(8):
        cmd, tick, done, nz, tg, te = st[r, :6]
        nxt = st[r + 1, 0] if r < 7 else 0.0
        pol = st[r + 1, 6] if r < 7 else 0.0
        w0n = st[r, 7]
        print("    %8.1f  roll %6.1f  fin %6.1f  noise %+6.1f  turn %6.1f  poll %+6.1f  wgend %+6.1f  tail %6.1f %6.1f" % (
            cmd, tick - cmd, done - tick, (nz - done) if nz else float("nan"), (nxt - done) if nxt else float("nan"),
            (pol - done) if pol else float("nan"), (w0n - done) if w0n else float("nan"),
            (tg - done) if tg else float("nan"), (te - tg) if te else float("nan")))
    eng.close()
    print(f"async_tail={async_tail}: " + "  ".join(f"[{i} step {a:.0f} out {b:.0f} L{l}]" for i, a, b, l in rows))
    print(f"  {n} back-to-back steps: {dt:.1f} us/step, launches {info['server_launches']}, steps {info['server_steps']}")
