"""GPU, world size 2 in two processes on ONE device: the product's K-sharded step end to end.

Each rank runs ``mppi_amd.distributed.ShardedMPPI`` (its shard's rollout + record on the
HIP engine, ``exchange_records``, the rank-order combine and the finish) with the record
exchange over gloo (RCCL refuses two ranks on one GPU; the driver's multi-GPU bench runs the
same code over RCCL).  Both ranks must emit identical controls and nominal sequences, equal
bit for bit to the one-process engine on the whole K (65536 per rank is a power-of-two leaf
count), over several steps of a closed loop on the nominal sequence.
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

STEPS = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from mppi_amd import scene
    return scene.scene_c3()


def _state(_lib):
    return _lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0)


def _worker(rank, world, port, K, H, q):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from mppi_amd import _lib
    from mppi_amd.distributed import ShardedMPPI
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Z, hw, cm = _scene()
        sh = ShardedMPPI(K, H, 0)
        sh.engine.set_dem(Z, hw)
        sh.engine.set_costmap(cm, hw)
        sh.engine.set_state(_state(_lib))
        outs = []
        for i in range(STEPS):
            o = sh.step("3d", i)
            outs.append({k: np.array(v, copy=True) for k, v in o.items()})
        torch.cuda.synchronize()
        q.put((rank, sh.k_begin, sh.k_count, outs))
        sh.close()
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_gpu_bitwise_equal_to_one_process():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    K, H = 2 * 65536, 100
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, K, H, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert [(r[1], r[2]) for r in res] == [(0, 65536), (65536, 65536)]

    from mppi_amd import _lib
    Z, hw, cm = _scene()
    eng = _lib.Engine(_lib.make_params(K, H), 0)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_state(_lib))
    for i in range(STEPS):
        one = eng.step("3d", i)
        for rank, _, _, outs in res:
            for key in ("u1_opt", "u2_opt", "lin_vel", "ang_vel"):
                np.testing.assert_array_equal(outs[i][key], one[key], err_msg=f"step {i} rank {rank} {key}")
            for key in ("traj_sim", "heading_sim"):  # row 0 arrives with the step (the rest with the tail)
                np.testing.assert_array_equal(outs[i][key][0], one[key][0], err_msg=f"step {i} rank {rank} {key}")
    eng.close()
