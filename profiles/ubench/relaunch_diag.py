"""Diagnostic (not part of the product): the cost of the first step after the resident server was
stopped (the bench's barrier stops it before the timed steps), C3 K 65536 H 100, deferred tail."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd"))
from mppi_amd import _lib, scene  # noqa: E402

Z, hw, cm = scene.scene_c3()
eng = _lib.Engine(_lib.make_params(65536, 100), 0)
eng.set_dem(Z, hw)
eng.set_costmap(cm, hw)
eng.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
eng.set_async_tail(True)
i = 0
for _ in range(50):
    eng.step("3d", i, copy=False)
    i += 1
for rep in range(6):
    eng.sync()
    ts = []
    for k in range(20):
        t0 = time.perf_counter()
        eng.step("3d", i, copy=False)
        ts.append((time.perf_counter() - t0) * 1e6)
        i += 1
    t0 = time.perf_counter()
    eng.outputs()
    tout = (time.perf_counter() - t0) * 1e6
    print("after sync: first %.1f  second %.1f  rest mean %.1f  max %.1f  final outputs() %.1f  total %.1f us" % (
        ts[0], ts[1], sum(ts[2:]) / 18, max(ts[2:]), tout, sum(ts) + tout))
print("launches", eng.launch_info()["server_launches"])
eng.close()
