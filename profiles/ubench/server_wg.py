"""Diagnostic (round 6): where the resident server's rollout spends its time at C3.  Runs back-to-back
server steps (deferred tails, or synchronous with --sync) and reads the last step's stamps: workgroup
0's chain clock (cycles per chain step on the server) and every workgroup's record time from the
first workgroup start (mppi_get_chain_clock out[10 + b]).
Usage (GPU box): python profiles/ubench/server_wg.py [steps] [--sync]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 200
    sync = "--sync" in sys.argv
    seed = int(os.environ.get("SEED", "42"))
    import torch  # noqa: F401
    from mppi_amd import _lib, scene
    Z, hw, cm = scene.scene_c3()
    eng = _lib.Engine(_lib.make_params(65536, 100, seed=seed), 0)
    eng.set_option("resident", 2)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
    eng.set_async_tail(not sync)
    for rep in range(3):
        for i in range(n):
            eng.step("3d", rep * n + i, copy=False)
        out = (C.c_double * (10 + 256))()
        assert eng.lib.mppi_get_chain_clock(eng.ctx, out, 10 + 256) == 0
        v = np.array(out[:])
        ends = v[10:10 + 256]
        order = np.argsort(ends)
        info = eng.launch_info()
        print(f"seed {seed} rep {rep} ({'sync' if sync else 'deferred tails'}): wg0 chain {v[1]:.1f} cycles/step at "
              f"{v[0]:.0f} MHz, chain {v[2]:.2f} us; wg start spread {v[7]:.2f} us, record ends "
              f"min {ends.min():.2f} median {np.median(ends):.2f} p90 {np.percentile(ends, 90):.2f} "
              f"max {ends.max():.2f} us; latest workgroups {order[-4:].tolist()} at "
              f"{[round(float(ends[b]), 2) for b in order[-4:]]}; wg0 record at {ends[0]:.2f}; "
              f"resident {info['resident']}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
