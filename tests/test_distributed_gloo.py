"""CPU, world_size 2 (gloo): the K-sharded protocol of mppi_amd.distributed.

Each rank computes its shard's softmax record with the oracle (the engine's
restatement), exchanges it with the product's ``exchange_records`` and combines
in rank order; the result must equal the one-rank step bit for bit when the
shards hold a power-of-two number of leaves, and be identical on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mppi_amd.distributed import LEAF, shard_bounds
from oracle import mppi_ref as R


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from mppi_amd import scene
    Z = scene.crater_dem(200, 10.0, [((-3.0, -4.0), 2.4, 3.1), ((4.0, 2.5), 3.2, 2.6)])
    cm = scene.disc_costmap(25, 10.0, scene.random_obstacles(n=10, seed=3, extent=8.0), power=10)
    return Z, 10.0, cm


def _worker(rank, world, port, K, H, q):
    import torch
    import torch.distributed as dist
    from mppi_amd.distributed import exchange_records
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Z, hw, cm = _scene()
        p = R.Params(K=K, H=H, seed=7)
        sc = R.Scene(Z, hw, cm)
        st = R.State(x=-5.0, y=1.0, goal_x=6.0, goal_y=-2.0)
        u = np.zeros(H, np.float32)
        b, c = shard_bounds(K, world)[rank]
        rec, _ = R.shard_record(p, sc, st, u, u, 2, b, c)
        E = 2 * H + 2
        mine = torch.from_numpy(rec.astype(np.float64))
        gathered = torch.empty(world * E, dtype=torch.float64)
        exchange_records(mine, gathered)
        recs = gathered.numpy().reshape(world, E)
        root = R.tree_reduce(recs, p.temperature)
        fin = R.finish(p, sc, st, root)
        q.put((rank, root, fin["u1_opt"], fin["u2_opt"], fin["v_opt"], fin["w_opt"]))
    finally:
        dist.destroy_process_group()


def _run(world, K, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, H, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_shard_bounds_match_oracle():
    for K in (1, 255, 256, 1000, 4096, 65536, 65536 * 8, 1 << 20):
        for world in (1, 2, 3, 4, 8):
            assert shard_bounds(K, world) == R.shard_bounds(K, world)
            bounds = shard_bounds(K, world)
            assert sum(c for _, c in bounds) == K
            assert all(b % LEAF == 0 for b, c in bounds if c > 0)


@pytest.mark.parametrize("K,H", [(1024, 12)])
def test_gloo_two_ranks_bitwise(K, H):
    res = _run(2, K, H)
    Z, hw, cm = _scene()
    p = R.Params(K=K, H=H, seed=7)
    st = R.State(x=-5.0, y=1.0, goal_x=6.0, goal_y=-2.0)
    u = np.zeros(H, np.float32)
    one = R.mppi_step(p, R.Scene(Z, hw, cm), st, u, u, 2)
    for rank, root, u1, u2, v, w in res:
        np.testing.assert_array_equal(root, one["root"], err_msg=f"rank {rank} root")
        np.testing.assert_array_equal(u1, one["u1_opt"])
        np.testing.assert_array_equal(u2, one["u2_opt"])
        np.testing.assert_array_equal(v, one["v_opt"])
        np.testing.assert_array_equal(w, one["w_opt"])


def test_gloo_ragged_shards_agree_across_ranks():
    """K not splitting into power-of-two leaf counts: still deterministic and equal on all ranks."""
    K, H = 700, 6
    res = _run(2, K, H)
    assert np.array_equal(res[0][1], res[1][1])
    Z, hw, cm = _scene()
    p = R.Params(K=K, H=H, seed=7)
    st = R.State(x=-5.0, y=1.0, goal_x=6.0, goal_y=-2.0)
    u = np.zeros(H, np.float32)
    sharded = R.mppi_step(p, R.Scene(Z, hw, cm), st, u, u, 2, world=2)
    np.testing.assert_array_equal(res[0][1], sharded["root"])
    one = R.mppi_step(p, R.Scene(Z, hw, cm), st, u, u, 2)
    rel = np.abs(sharded["u1_opt"] - one["u1_opt"]) / np.maximum(np.abs(one["u1_opt"]), 1e-3)
    assert rel.max() <= 1e-5


class _OracleEngine:
    """CPU stand-in for the HIP engine behind ShardedMPPI: the same three calls, computed by the
    oracle (record of this rank's slice; finish over the gathered records)."""

    def __init__(self, K, H, k_offset, K_global, sharded_ref):
        self.K, self.H, self.k0, self.K_global = K, H, k_offset, K_global
        self.sh = sharded_ref
        self.partial_calls = 0

    def record_len(self):
        return 2 * self.H + 2

    def _setup(self):
        Z, hw, cm = _scene()
        p = R.Params(K=self.K_global, H=self.H, seed=7)
        return p, R.Scene(Z, hw, cm), R.State(x=-5.0, y=1.0, goal_x=6.0, goal_y=-2.0)

    def step_partial(self, ptr, proj, step):
        import torch
        self.partial_calls += 1
        p, sc, st = self._setup()
        u = np.zeros(self.H, np.float32)
        rec, _ = R.shard_record(p, sc, st, u, u, step, self.k0, self.K)
        sh = self.sh[0]
        assert ptr == sh.record.data_ptr()
        sh.record.copy_(torch.from_numpy(rec))

    def step_finish(self, ptr, n, copy=True):
        sh = self.sh[0]
        assert ptr == sh.gathered.data_ptr() and n == sh.world
        p, sc, st = self._setup()
        recs = sh.gathered.numpy().reshape(n, -1)
        root = R.tree_reduce(recs, p.temperature)
        out = R.finish(p, sc, st, root)
        out["root"] = root
        return out

    def close(self):
        pass


def _sharded_worker(rank, world, port, K, H, q):
    import torch.distributed as dist
    from mppi_amd.distributed import ShardedMPPI
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        holder = []
        eng = []

        def factory(k, h, k0, device):
            e = _OracleEngine(k, h, k0, K, holder)
            eng.append(e)
            return e

        sh = ShardedMPPI(K, H, "cpu", engine_factory=factory)
        holder.append(sh)
        out = sh.step("3d", 2)
        q.put((rank, sh.empty, eng[0].partial_calls, out["root"], out["u1_opt"], out["v_opt"]))
        sh.close()
    finally:
        dist.destroy_process_group()


def test_gloo_sharded_mppi_with_empty_shard():
    """ShardedMPPI's own exchange (world 4, K=1280: rank 3 owns no trajectory).  The empty rank
    contributes the empty record and no rank blocks; every rank emits the one-rank result's
    controls, and the root equals the oracle's 4-shard combine."""
    world, K, H = 4, 1280, 6
    assert shard_bounds(K, world)[3] == (1280, 0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, K, H, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    Z, hw, cm = _scene()
    p = R.Params(K=K, H=H, seed=7)
    st = R.State(x=-5.0, y=1.0, goal_x=6.0, goal_y=-2.0)
    u = np.zeros(H, np.float32)
    sharded = R.mppi_step(p, R.Scene(Z, hw, cm), st, u, u, 2, world=world)
    for rank, empty, calls, root, u1, v in res:
        assert empty == (rank == 3)
        assert calls == (0 if rank == 3 else 1)
        np.testing.assert_array_equal(root, sharded["root"])
        np.testing.assert_array_equal(u1, sharded["u1_opt"])
        np.testing.assert_array_equal(v, sharded["v_opt"])
