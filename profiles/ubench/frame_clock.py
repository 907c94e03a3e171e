"""Diagnostic (round 6): the rollout's shader clock and chain cycles at a simulator frame cadence
(separate launches, with and without the bench's stand-in between frames) against back-to-back
steps.  Usage (GPU box): python profiles/ubench/frame_clock.py"""
import os
import sys
import time

import numpy as np

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
    step = 0
    for rep in range(2):
        for mode in ("b2b", "frame", "frame+standin", "frame16+standin"):
            rows = []
            for f in range(15):
                if mode == "b2b":
                    for _ in range(5):
                        e.step("3d", step, copy=False)
                        step += 1
                else:
                    gap = 16e-3 if mode.startswith("frame16") else 2e-3
                    if mode.endswith("standin"):
                        with torch.cuda.stream(sim):
                            dst.copy_(src)
                            torch.matmul(A, B)
                        sim.synchronize()
                    t1 = time.perf_counter()
                    while time.perf_counter() - t1 < gap:
                        time.sleep(0.0002)
                    t0 = time.perf_counter()
                    e.step("3d", step, copy=False)
                    lat = (time.perf_counter() - t0) * 1e6
                    step += 1
                c = e.chain_clock()
                rows.append((c["shader_mhz"], c["cycles_per_step"], c["chain_us"], c["leaf_us"],
                             c["wg_start_spread_us"], c["wg_span_us"], lat if mode != "b2b" else 0.0))
            m = np.median(np.array(rows), axis=0)
            print(f"rep {rep} {mode}: shader {m[0]:.0f} MHz, chain {m[1]:.0f} cycles/step = {m[2]:.1f} us, leaf {m[3]:.1f} "
                  f"us, wg start spread {m[4]:.1f} us, span {m[5]:.1f} us, call latency {m[6]:.1f} us", flush=True)
    e.close()


if __name__ == "__main__":
    main()
