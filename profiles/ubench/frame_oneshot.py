"""Diagnostic (round 6): at a simulator frame cadence, one step as separate launches (rollout, finish)
against one step on a server launch that leaves right after it (mppi_set_option "server_exit_after"
1 before every step: no idle period) and against the server relaunched per frame with its idle limit
(resident 2).  Per frame: step, the bench's stand-in (1 GiB copy + bf16 GEMM, waited for), rest of the
gap.  Usage (GPU box): python profiles/ubench/frame_oneshot.py [rounds]"""
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
    st = _lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0)
    Z, hw, cm = scene.scene_c3()
    dev = torch.device("cuda", 0)
    src = torch.ones(1 << 28, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    A = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    B = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    sim = torch.cuda.Stream(device=dev)

    def world_step():
        with torch.cuda.stream(sim):
            dst.copy_(src)
            torch.matmul(A, B)
        sim.synchronize()

    outs = {}
    for K in (65536, 1000):
        for gap in (2.0, 16.0):
            for r in range(rounds):
                for sched in ("separate", "oneshot", "server"):
                    e = _lib.Engine(_lib.make_params(K, 100), 0)
                    e.set_option("resident", 0 if sched == "separate" else 2)
                    e.set_dem(Z, hw)
                    e.set_costmap(cm, hw)
                    e.set_state(st)
                    e.set_async_tail(True)
                    for i in range(10):
                        e.step("3d", i, copy=False)
                    lat, seq = [], []
                    for f in range(40):
                        if sched == "oneshot":
                            e.set_option("server_exit_after", 1)
                        t0 = time.perf_counter()
                        o = e.step("3d", 10 + f)
                        t1 = time.perf_counter()
                        seq.append(o["u1_opt"].copy())
                        lat.append((t1 - t0) * 1e6)
                        world_step()
                        while (time.perf_counter() - t1) * 1e3 < gap:
                            time.sleep(0.0002)
                    info = e.launch_info()
                    e.close()
                    if r == 0 and gap == 2.0:
                        outs[(K, sched)] = np.stack(seq)
                    print(f"round {r} K={K} gap {gap} ms {sched}: p50 {np.median(lat):.1f} us p90 "
                          f"{np.percentile(lat, 90):.1f} us, launches {info['server_launches']}, "
                          f"server steps {info['server_steps']}", flush=True)
        print(f"K={K} bitwise oneshot/server vs separate:",
              np.array_equal(outs[(K, 'oneshot')], outs[(K, 'separate')]),
              np.array_equal(outs[(K, 'server')], outs[(K, 'separate')]), flush=True)


if __name__ == "__main__":
    main()
