"""GPU: the K-sharded step's RCCL exchange on the engine stream (mppi_amd.distributed).

RCCL refuses two ranks on one GPU, so this runs ONE rank over the ``nccl`` backend (RCCL on
ROCm) with ``always_exchange=True``: partial step (rollout + the rank's record) on the engine's
torch stream -> ``dist.all_gather_into_tensor`` on that stream -> the rank-order finish.  The
outputs must equal the one-context engine bit for bit over a closed loop of steps.  (The
multi-rank exchange itself is covered by gloo on CPU and by the driver's 8-GPU bench.)
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")

pytestmark = pytest.mark.gpu

KEYS = ("u1_opt", "u2_opt", "lin_vel", "ang_vel", "traj_sim")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, K, H, steps, q):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from mppi_amd import _lib, scene
    from mppi_amd.distributed import ShardedMPPI
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        Z, hw, cm = scene.scene_c3()
        st = _lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0)
        sh = ShardedMPPI(K, H, 0, always_exchange=True)
        one = _lib.Engine(_lib.make_params(K, H), 0)
        for e in (sh.engine, one):
            e.set_dem(Z, hw)
            e.set_costmap(cm, hw)
            e.set_state(st)
        bad = []
        for i in range(steps):
            a = sh.step("3d", i)
            b = one.step("3d", i)
            for k in KEYS:
                if not np.array_equal(a[k], b[k]):
                    bad.append(f"step {i} {k}")
        backend = dist.get_backend()
        sh.close()
        one.close()
        q.put((backend, bad))
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_one_rank_bitwise():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_worker, args=(_free_port(), 65536, 24, 3, q))
    pr.start()
    backend, bad = q.get(timeout=240)
    pr.join(timeout=60)
    assert pr.exitcode == 0
    assert backend == "nccl"
    assert not bad, bad
