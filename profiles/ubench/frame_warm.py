"""Diagnostic (round 6, for the experiment build only: the "warm" option and its warm-up code were removed
after this measurement, profiles/r06_notes.md): the role-split rollout's cache warm-up at a frame
cadence beside the bench's simulator stand-in (1 GiB copy + bf16 GEMM, waited for), alternating
warm 0 / 1: call latency p50 / p90, the chain's cycles per step; and back to back (separate launches,
warm 0 / 2).  Usage (GPU box): python profiles/ubench/frame_warm.py [rounds]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import torch
    from mppi_amd import _lib, scene
    Z, hw, cm = scene.scene_c3()
    dev = torch.device("cuda", 0)
    src = torch.ones(1 << 28, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    A = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    B = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    sim = torch.cuda.Stream(device=dev)
    st = _lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0)

    def world():
        with torch.cuda.stream(sim):
            dst.copy_(src)
            torch.matmul(A, B)
        sim.synchronize()

    for K in (65536, 1000):
        for gap in (2e-3, 16e-3):
            for r in range(rounds):
                for warm in (0, 1):
                    e = _lib.Engine(_lib.make_params(K, 100), 0)
                    e.set_option("warm", warm)
                    e.set_dem(Z, hw)
                    e.set_costmap(cm, hw)
                    e.set_state(st)
                    e.set_async_tail(True)
                    for i in range(10):
                        e.step("3d", i, copy=False)
                    lat, cyc = [], []
                    for f in range(30):
                        world()
                        t1 = time.perf_counter()
                        while time.perf_counter() - t1 < gap:
                            time.sleep(0.0002)
                        t0 = time.perf_counter()
                        e.step("3d", 10 + f, copy=False)
                        lat.append((time.perf_counter() - t0) * 1e6)
                        if f % 3 == 2:
                            cyc.append(e.chain_clock()["cycles_per_step"])
                    e.close()
                    print(f"round {r} K={K} gap {gap * 1e3:.0f} ms warm={warm}: p50 {np.median(lat):.1f} us p90 "
                          f"{np.percentile(lat, 90):.1f} us, chain {np.median(cyc):.0f} cycles/step", flush=True)
    e = _lib.Engine(_lib.make_params(65536, 100), 0)
    e.set_option("resident", 0)
    e.set_dem(Z, hw)
    e.set_costmap(cm, hw)
    e.set_state(st)
    e.set_async_tail(True)
    step = 0
    for r in range(rounds):
        for warm in (0, 2):
            e.set_option("warm", warm)
            for _ in range(20):
                e.step("3d", step, copy=False)
                step += 1
            e.outputs()
            t0 = time.perf_counter()
            for _ in range(200):
                e.step("3d", step, copy=False)
                step += 1
            e.outputs()
            print(f"round {r} back-to-back separate launches warm={warm}: "
                  f"{(time.perf_counter() - t0) / 200 * 1e6:.1f} us/step", flush=True)
    e.close()


if __name__ == "__main__":
    main()
