"""GPU: the HIP engine reproduces the committed golden step vectors (tests/golden/step_small.npz) bit for bit,
and the K-sharded partial/finish ABI is shard-invariant on one device."""
import importlib.util
import os

import numpy as np
import pytest

import helpers as hp
from oracle import mppi_ref as R

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _make_golden():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLD, "step_small.npz")) as f:
        return {k: f[k] for k in f.files}


@pytest.mark.parametrize("name", ["far3d", "near3d", "twod", "ragged", "injected"])
def test_engine_matches_golden_vectors(gold, name):
    from mppi_amd import _lib
    mg = _make_golden()
    K, H, proj, step, start, heading, wheels, goal, sigma, nom_seed, inj = mg.STEP_CASES[name]
    eng = _lib.Engine(_lib.make_params(K, H, seed=42), 0)
    eng.set_dem(gold["Z"], float(gold["hw"]))
    eng.set_costmap(gold["cm"], float(gold["hw"]))
    eng.set_state(_lib.make_state(start[0], start[1], heading, wheels[0], wheels[1], goal[0], goal[1],
                                  sigma[0], sigma[1]))
    eng.set_nominal(gold[f"{name}/u_nom1"], gold[f"{name}/u_nom2"])
    if inj:
        out = eng.step_injected(gold[f"{name}/inj_u1"], gold[f"{name}/inj_u2"], proj)
    else:
        out = eng.step(proj, step)
    g = lambda k: gold[f"{name}/{k}"]  # noqa: E731
    assert np.array_equal(eng.costs(), g("cost")), hp.mismatch_report("cost", eng.costs(), g("cost"))
    for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt"),
                 ("traj_sim", "traj_sim"), ("heading_sim", "hv_sim"), ("left_wheel_sim", "lw_sim"),
                 ("right_wheel_sim", "rw_sim")):
        assert np.array_equal(out[a], g(b)), hp.mismatch_report(a, out[a], g(b))
    eng.close()


@pytest.mark.parametrize("K,H,world", [(4096, 50, 2), (8192, 30, 4), (1000, 20, 2)])
def test_partial_finish_shards_on_one_gpu(K, H, world):
    """Per-shard engines (k_offset = shard begin) + records gathered in rank order == one-engine step."""
    import torch
    from mppi_amd import _lib
    from mppi_amd.distributed import shard_bounds
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(wl=0.2, wr=0.4)
    engines = []
    for b, c in shard_bounds(K, world):
        e = hp.engine_for(c, H, Z, hw, cm, st, seed=3, k_offset=b)
        engines.append(e)
    E = engines[0].record_len()
    assert E == 2 * H + 2
    recs = torch.empty(world * E, dtype=torch.float64, device="cuda:0")
    for g, e in enumerate(engines):
        e.step_partial(recs[g * E:(g + 1) * E].data_ptr(), "3d", 4)
    torch.cuda.synchronize()
    outs = [e.step_finish(recs.data_ptr(), world) for e in engines]
    ref = R.mppi_step(R.Params(K=K, H=H, seed=3), hp.oracle_scene(Z, hw, cm), st, np.zeros(H, np.float32),
                      np.zeros(H, np.float32), 4, world=world)
    np.testing.assert_array_equal(recs.cpu().numpy().reshape(world, E),
                                  np.stack([R.tree_reduce(R.leaf_records(p["cost"], p["u1"], p["u2"], 0.3), 0.3)
                                            for p in ref["parts"]]))
    for o in outs:     # every rank emits the same controls
        for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt"),
                     ("traj_sim", "traj_sim")):
            assert np.array_equal(o[a], ref[b]), hp.mismatch_report(a, o[a], ref[b])
    pow2 = all((c // 256) & ((c // 256) - 1) == 0 and c % 256 == 0 for _, c in shard_bounds(K, world))
    if pow2:   # shard-invariant bit for bit against the single-engine step
        one = hp.engine_for(K, H, Z, hw, cm, st, seed=3).step("3d", 4)
        for a in ("u1_opt", "u2_opt", "lin_vel", "ang_vel", "traj_sim"):
            assert np.array_equal(outs[0][a], one[a]), a
    for e in engines:
        e.close()


@pytest.mark.parametrize("proj", ["3d", "2d"])
def test_async_tail_bitwise_equal_to_sync(proj):
    """Deferred optimal rollout: controls + row 0 at return, all rows after outputs(); identical to sync mode."""
    K, H = 2048, 40
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(wl=0.3, wr=0.5)
    sync = hp.engine_for(K, H, Z, hw, cm, st, seed=9)
    asyn = hp.engine_for(K, H, Z, hw, cm, st, seed=9)
    asyn.set_async_tail(True)
    for i in range(4):          # nominal chain across steps, tails overlapping the next rollout
        a = asyn.step(proj, i)
        b = sync.step(proj, i)
        for k in ("u1_opt", "u2_opt", "lin_vel", "ang_vel"):
            assert np.array_equal(a[k], b[k]), (i, k)
        for k in ("traj_sim", "heading_sim", "left_wheel_sim", "right_wheel_sim"):
            assert np.array_equal(a[k][0], b[k][0]), (i, k, "row 0")
        if i % 2 == 1:
            full = asyn.outputs()
            for k in b:
                assert np.array_equal(full[k], b[k]), (i, k)
    # a DEM change waits for the in-flight tail; the next step sees the new terrain
    asyn.set_dem(Z * 2.0, hw)
    sync.set_dem(Z * 2.0, hw)
    a = asyn.step(proj, 7)
    b = sync.step(proj, 7)
    full = asyn.outputs()
    for k in b:
        assert np.array_equal(full[k], b[k]), k
    t_ms, n = asyn.tail_timing()
    assert n == 0 or t_ms > 0
