"""Diagnostic (round 6): one C3 step per 2 ms frame as separate launches (the default schedule at a
frame cadence) beside the bench's simulator stand-in, with the host's CLOCK_MONOTONIC stamps of every
call's entry and return (stdout), for alignment with a rocprofv3 kernel trace of the same run.
Usage (GPU box): rocprofv3 --kernel-trace -d DIR -o k --output-format csv -- python3 frame_trace.py > stamps"""
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
    e.set_dem(Z, hw)
    e.set_costmap(cm, hw)
    e.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
    e.set_async_tail(True)
    for i in range(10):
        e.step("3d", i, copy=False)
    for f in range(40):
        t0 = time.monotonic_ns()
        e.step("3d", 10 + f, copy=False)
        t1 = time.monotonic_ns()
        print(f"frame {f} {t0} {t1}", flush=True)
        with torch.cuda.stream(sim):
            dst.copy_(src)
            torch.matmul(A, B)
        sim.synchronize()
        while (time.monotonic_ns() - t1) < 2_000_000:
            time.sleep(0.0002)
    print("info", e.launch_info(), flush=True)
    e.close()


if __name__ == "__main__":
    main()
