"""GPU: the 8-way K split each GPU of the 8-GPU runs performs, at FULL size.

An 8-member mppi_group on device 0 runs exactly the per-GPU work of the 8-GPU C4 and C5 runs:
every member rolls out its 1/8 of K, reduces it to one (m, S, V1[H], V2[H]) record, and every
member combines the 8 records in member order and runs the finish.  Members sharing a device
exchange the records by device copies; on distinct devices the same 8 records travel by
ncclAllGather (the combine and the finish are the same code).

* C4: K = 1,048,576, H = 100 -> 131,072 trajectories (512 leaves) per member.
* C5: K = 262,144, H = 128 on the 8192^2 DEM -> 32,768 trajectories (128 leaves) per member.

Both are power-of-two leaf splits, so the member roots are subtrees of the one-context tree and
three chained steps are bitwise equal to one context over all K (which reduces 4096 / 1024 leaf
records in one finish).  Step 0 is also checked against the oracle's world=8 combine (shard
records in member order, `R.tree_reduce`), the emitted controls bit-exact and within 1e-5.
Reference: critics_warp.py:338-376 (weights, sums), MPPI_isaac.py:632-720 (update, tail).
"""
import functools

import numpy as np
import pytest

import helpers as hp
from oracle import mppi_ref as R

pytestmark = pytest.mark.gpu

TOL = 1e-5
N = 8
OUTS = ("u1_opt", "u2_opt", "lin_vel", "ang_vel", "traj_sim", "heading_sim", "left_wheel_sim",
        "right_wheel_sim")
REF = dict(u1_opt="u1_opt", u2_opt="u2_opt", lin_vel="v_opt", ang_vel="w_opt", traj_sim="traj_sim",
           heading_sim="hv_sim", left_wheel_sim="lw_sim", right_wheel_sim="rw_sim")


@functools.lru_cache(maxsize=1)
def _c5_scene():
    from mppi_amd import scene
    return scene.scene_c5()


def _oracle_world(p, sc, st, step, chunk):
    """The oracle's world=N step: each member's record from `chunk`-sized pieces of its shard
    (power-of-two leaf counts, so the pieces' roots are the shard tree's subtrees), the member
    roots combined in member order, then the finish."""
    u = np.zeros(p.H, np.float32)
    roots, costs = [], []
    for b, c in R.shard_bounds(p.K, N):
        parts = []
        for o in range(b, b + c, chunk):
            rec, part = R.shard_record(p, sc, st, u, u, step, o, min(chunk, b + c - o))
            parts.append(rec)
            costs.append(part["cost"])
            del part
        roots.append(R.tree_reduce(np.stack(parts), p.temperature) if len(parts) > 1 else parts[0])
    ref = R.finish(p, sc, st, R.tree_reduce(np.stack(roots), p.temperature))
    ref["cost"] = np.concatenate(costs)
    return ref


def _run(K, H, Z, hw, cm, st, seed, chunk, async_tail):
    from mppi_amd import _lib
    p = R.Params(K=K, H=H, seed=seed)
    ref = _oracle_world(p, R.Scene(Z, hw, cm), st, 0, chunk)
    one = hp.engine_for(K, H, Z, hw, cm, st, seed=seed)
    g = _lib.Group(_lib.make_params(K, H, seed=seed), [0] * N)
    try:
        g.set_dem(Z, hw)
        g.set_costmap(cm, hw)
        g.set_state(hp.state_for(st))
        assert [g.shard(i) for i in range(N)] == R.shard_bounds(K, N)
        assert all(g.shard(i)[1] == K // N for i in range(N))
        if async_tail:
            g.set_async_tail(True)
            one.set_async_tail(True)
        for it in range(3):
            go = g.step("3d", it)
            oo = one.step("3d", it)
            if async_tail:
                go, oo = g.outputs(), one.outputs()
            for k in OUTS:
                assert np.array_equal(go[k], oo[k]), f"step {it}: " + hp.mismatch_report(k, go[k], oo[k])
            gc = g.costs()
            assert np.array_equal(gc, one.costs()), f"step {it}: costs differ"
            if it == 0:
                assert np.array_equal(gc, ref["cost"]), hp.mismatch_report("cost", gc, ref["cost"])
                for k in OUTS:
                    assert np.array_equal(go[k], ref[REF[k]]), hp.mismatch_report(k, go[k], ref[REF[k]])
                for k in ("u1_opt", "u2_opt", "lin_vel", "ang_vel"):
                    assert hp.rel_err(go[k], ref[REF[k]]) <= TOL
        # every member ends on the same nominal controls as the one context
        u1, u2 = one.get_nominal()
        for m in g.members:
            a1, a2 = m.get_nominal()
            assert np.array_equal(a1, u1) and np.array_equal(a2, u2)
    finally:
        g.close()
        one.close()


def test_group8_c4_full_size():
    """C4: 8 members x 131,072 trajectories, H = 100, on device 0 (the per-GPU work of the
    8-GPU C4 run); three chained steps bitwise equal to one 1,048,576-trajectory context."""
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(wl=0.05, wr=0.1)
    _run(1048576, 100, Z, hw, cm, st, seed=7, chunk=65536, async_tail=False)


def test_group8_c5_full_size():
    """C5: 8 members x 32,768 trajectories, H = 128, 8192^2 DEM @0.025 m; the deferred optimal
    rollout on (the bench's schedule); bitwise equal to one 262,144-trajectory context."""
    Z, hw, cm = _c5_scene()
    st = hp.oracle_state(x=0.0, y=0.0, goal=(80.0, 20.0), wl=0.2, wr=0.3)
    _run(262144, 128, Z, hw, cm, st, seed=42, chunk=32768, async_tail=True)
