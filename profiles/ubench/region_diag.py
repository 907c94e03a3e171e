"""Diagnostic (not part of the product): where the bench's fixed per-region cost goes.  The bench's
timed region (bench.py timed_run) starts with the resident server stopped (mppi_sync + synchronize)
and ends with the last step's deferred optimal rollout, the server's stop and a synchronize.  Here:
W warm-up steps, then R regions of N steps at C3; per region the wall time of the first step call,
the mean of the other step calls, the final outputs() wait and the sync (server stop), in us."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd"))
import torch  # noqa: E402
from mppi_amd import _lib, scene  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 6
Z, hw, cm = scene.scene_c3()
eng = _lib.Engine(_lib.make_params(65536, 100), 0)
eng.set_dem(Z, hw)
eng.set_costmap(cm, hw)
eng.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
eng.set_async_tail(True)
for i in range(5):
    eng.step("3d", i, copy=False)
step = 5
for r in range(R):
    eng.sync()
    torch.cuda.synchronize()
    t = [time.perf_counter()]
    for i in range(N):
        eng.step("3d", step, copy=False)
        step += 1
        t.append(time.perf_counter())
    eng.outputs()
    t.append(time.perf_counter())
    eng.sync()
    t.append(time.perf_counter())
    torch.cuda.synchronize()
    t.append(time.perf_counter())
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"  second cuda sync {(t2 - t[-1]) * 1e6:.1f}")
    us = [(b - a) * 1e6 for a, b in zip(t, t[1:])]
    total = (t[-1] - t[0]) * 1e6
    first, rest, outs, stop, cs = us[0], us[1:N], us[N], us[N + 1], us[N + 2]
    print(f"region {r}: total {total:.0f} us ({N / total * 1e6:.0f} steps/s)  first step {first:.1f}  "
          f"steps 2..{N} mean {sum(rest) / len(rest):.1f} (2nd {rest[0]:.1f}, 3rd {rest[1]:.1f})  "
          f"outputs {outs:.1f}  stop {stop:.1f}  cuda sync {cs:.1f}  launches {eng.launch_info()['server_launches']}")
# the stop alone: an idle server (no tail, no noise in flight), stopped 20 us / 150 us after its last step
for gap in (20e-6, 150e-6):
    for r in range(3):
        eng.step("3d", step, copy=False)
        step += 1
        eng.outputs()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < gap:
            pass
        t1 = time.perf_counter()
        eng.sync()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(f"idle {gap * 1e6:.0f} us: stop {(t2 - t1) * 1e6:.1f}  cuda sync {(t3 - t2) * 1e6:.1f}")
eng.close()
