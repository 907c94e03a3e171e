"""Diagnostic (round 6): where the next steps' normals are ordered on the separate-launch
path: after the rollout (eps_after 0: an event marker between the rollout and the finish on the context
stream), after the finish (1: no marker between them) or by the call's cadence (-1, the default).
Alternating on one box: C3 back-to-back separate launches (resident 0) and C3 at a 2 ms frame cadence
(p50 call latency); bitwise: the same steps' outputs under 0 and 1.  (Round 6's first run also timed
the C4 shard step, partial -> 1-rank RCCL all-gather -> finish: 168.6-173.6 us with 0, 178.0-179.0
with 1, profiles/r06_notes.md.)
Usage (GPU box): python profiles/ubench/eps_after_ab.py [rounds]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch
    from mppi_amd import _lib, scene
    st = _lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0)
    Z, hw, cm = scene.scene_c3()

    # bitwise: outputs of the same steps under both orders (separate launches, async tails)
    outs = []
    for ea in (0, 1):
        e = _lib.Engine(_lib.make_params(65536, 100), 0)
        e.set_option("resident", 0)
        e.set_option("eps_after", ea)
        e.set_dem(Z, hw)
        e.set_costmap(cm, hw)
        e.set_state(st)
        e.set_async_tail(True)
        seq = []
        for i in range(6):
            e.step("3d", i, copy=False)
            seq.append(np.concatenate([np.asarray(v, np.float32).ravel() for v in e.outputs().values()
                                       if isinstance(v, np.ndarray)]))
        e.close()
        outs.append(np.stack(seq))
    print("bitwise (6 steps, all outputs):", bool(np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))),
          flush=True)

    # C3 separate launches: back to back and at a 2 ms cadence
    e = _lib.Engine(_lib.make_params(65536, 100), 0)
    e.set_option("resident", 0)
    e.set_dem(Z, hw)
    e.set_costmap(cm, hw)
    e.set_state(st)
    e.set_async_tail(True)
    step = 0
    for r in range(rounds):
        for ea in (0, -1):
            e.set_option("eps_after", ea)
            for _ in range(20):
                e.step("3d", step, copy=False)
                step += 1
            e.outputs()
            t0 = time.perf_counter()
            for _ in range(200):
                e.step("3d", step, copy=False)
                step += 1
            e.outputs()
            bb = (time.perf_counter() - t0) / 200 * 1e6
            lat = []
            for _ in range(60):
                t0 = time.perf_counter()
                e.step("3d", step, copy=False)
                t1 = time.perf_counter()
                step += 1
                lat.append((t1 - t0) * 1e6)
                while (time.perf_counter() - t1) < 2e-3:
                    time.sleep(0.0002)
            e.outputs()
            print(f"round {r} eps_after={ea}: C3 separate back-to-back {bb:.1f} us/step, 2 ms cadence p50 "
                  f"{np.median(lat):.1f} us p90 {np.percentile(lat, 90):.1f} us", flush=True)
    e.close()

    # at the bench's cadence (bench.py cadence_bench): step, then a simulator-frame stand-in on its own
    # stream (1 GiB copy + bf16 4096^3 GEMM) waited for, then the rest of the frame gap
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

    for K in (65536, 1000):
        for gap in (2.0, 16.0):
            for r in range(rounds):
                for ea in (0, -1):
                    e = _lib.Engine(_lib.make_params(K, 100), 0)
                    e.set_option("resident", 0)
                    e.set_option("eps_after", ea)
                    e.set_dem(Z, hw)
                    e.set_costmap(cm, hw)
                    e.set_state(st)
                    e.set_async_tail(True)
                    for i in range(10):
                        e.step("3d", i, copy=False)
                    lat = []
                    for f in range(40):
                        t0 = time.perf_counter()
                        e.step("3d", 10 + f, copy=False)
                        t1 = time.perf_counter()
                        lat.append((t1 - t0) * 1e6)
                        world_step()
                        while (time.perf_counter() - t1) * 1e3 < gap:
                            time.sleep(0.0002)
                    e.close()
                    print(f"round {r} K={K} gap {gap} ms eps_after={ea}: with the stand-in p50 {np.median(lat):.1f} us "
                          f"p90 {np.percentile(lat, 90):.1f} us", flush=True)


if __name__ == "__main__":
    main()
