"""Diagnostic (not part of the product): the plain one-context step at K = 131 072 (the C4 shard's
size) before and after the bench's bilinear leg, for an engine created before it, one created after
it, and one created after torch.cuda.empty_cache()."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from mppi_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
K, H, scene_fn, start, goal, _ = bench.CONFIGS["c4s8"]
Z, hw, cm = bench.get_scene(scene_fn)
state = _lib.make_state(start[0], start[1], (1.0, 0.0, 0.0), goal_x=goal[0], goal_y=goal[1])


def mk():
    e = _lib.Engine(_lib.make_params(K, H), 0)
    e.set_dem(Z, hw)
    e.set_costmap(cm, hw)
    e.set_state(state)
    e.set_async_tail(True)
    return e


def rate(e, tag, steps=200, warm=20):
    for i in range(warm):
        e.step("3d", i, copy=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        e.step("3d", warm + i, copy=False)
    e.outputs()
    torch.cuda.synchronize()
    print(f"{tag}: {(time.perf_counter() - t0) / steps * 1e3:.4f} ms per step", flush=True)


a = mk()
rate(a, "engine A before the bilinear leg")
print("bilinear:", bench.bilinear_bench(torch, dev)["kernel_avg_ms"], flush=True)
rate(a, "engine A after")
b = mk()
rate(b, "engine B created after")
b.close()
a.close()
torch.cuda.empty_cache()
c = mk()
rate(c, "engine C after empty_cache")
c.close()
