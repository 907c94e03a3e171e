"""Diagnostic (round 6): the same C3 separate-launch rollout back to back (30 steps) and then at a 2 ms
frame cadence after the bench's simulator stand-in (20 steps), for a rocprofv3 --pmc pass: the
roles-kernel rows in dispatch order are 30 back-to-back launches, then 20 frame-cadence ones.
Usage (GPU box): rocprofv3 --pmc <counters> --kernel-trace -d DIR -o p --output-format csv -- python3 frame_pmc.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]


def main():
    import torch
    from mppi_amd import _lib, scene
    Z, hw, cm = scene.scene_c3()
    dev = torch.device("cuda", 0)
    src = torch.ones(1 << 28, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    A = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    B = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    sim = torch.cuda.Stream(device=dev)
    e = _lib.Engine(_lib.make_params(65536, 100), 0)
    e.set_option("resident", 0)
    e.set_dem(Z, hw)
    e.set_costmap(cm, hw)
    e.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
    e.set_async_tail(True)
    for i in range(30):
        e.step("3d", i, copy=False)
    e.outputs()
    for f in range(20):
        with torch.cuda.stream(sim):
            dst.copy_(src)
            torch.matmul(A, B)
        sim.synchronize()
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < 2e-3:
            time.sleep(0.0002)
        e.step("3d", 30 + f, copy=False)
    e.outputs()
    e.close()
    print("done", flush=True)


if __name__ == "__main__":
    main()
