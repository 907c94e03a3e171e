"""Diagnostic: per-GPU step time of the K-sharded path (partial -> RCCL all-gather -> finish) on one
GPU with the exchange forced (world size 1, nccl backend), against the plain one-context step.
Usage (GPU box): python profiles/ubench/shard_step.py [K] [H] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    import torch
    import torch.distributed as dist
    from mppi_amd import _lib, scene
    from mppi_amd.distributed import ShardedMPPI
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    Z, hw, cm = scene.scene_c3()
    st = _lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0)
    sh = ShardedMPPI(K, H, 0, always_exchange=True)
    one = _lib.Engine(_lib.make_params(K, H), 0)
    for e in (sh.engine, one):
        e.set_dem(Z, hw)
        e.set_costmap(cm, hw)
        e.set_state(st)
        e.set_async_tail(True)
    for name, fn in (("plain", lambda i: one.step("3d", i, copy=False)),
                     ("sharded", lambda i: sh.step("3d", i, copy=False))):
        for i in range(20):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn(20 + i)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        print(f"K={K} H={H} {name}: {dt * 1e6:.1f} us/step ({1 / dt:.0f} steps/s)")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
