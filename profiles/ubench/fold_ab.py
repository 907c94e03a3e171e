"""Diagnostic (round 6): the C4 shard step (K = 131 072 per GPU: partial step -> 1-rank RCCL all-gather ->
finish, a one-member C-ABI group with the exchange forced) with the rank record's finish folded into the
rollout kernel (mppi_set_option "fold_record" 1) and as its own launch (0), alternating.
Usage (GPU box, a build of branch fold-record-wip, where the option exists): python profiles/ubench/fold_ab.py
[rounds] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    import torch
    from mppi_amd import _lib, scene
    os.environ["MPPI_GROUP_RCCL"] = "1"
    K, H = 131072, 100
    Z, hw, cm = scene.scene_c3()
    st = _lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0)
    g = _lib.Group(_lib.make_params(K, H), [0])
    e = g.members[0]
    e.set_dem(Z, hw)
    e.set_costmap(cm, hw)
    e.set_state(st)
    e.set_async_tail(True)
    step = 0
    for r in range(rounds):
        for fold in (1, 0):
            e.set_option("fold_record", fold)
            for _ in range(20):
                g.step("3d", step, copy=False)
                step += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                g.step("3d", step, copy=False)
                step += 1
            g.outputs()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            print(f"round {r} fold={fold}: {dt * 1e6:.1f} us/step, finish kind {e.launch_info()['finish_kind']}",
                  flush=True)
    g.close()


if __name__ == "__main__":
    main()
