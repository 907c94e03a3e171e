"""HIP engine vs the numpy restatement (oracle/), through the C-ABI.

Bar (BASELINE.json north_star): emitted control vector within 1e-5 relative
(max |a-b| / max(|ref|, 1e-3)).  Because every float op and transcendental is
defined identically on both sides, costs and rollouts are expected BIT-EXACT
and the tests assert that too; the 1e-5 check is the documented tolerance.
"""
import numpy as np
import pytest

import helpers as hp
from oracle import mppi_ref as R

TOL = 1e-5

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["roles", "pair"])
def rollout_kernel(request, monkeypatch):
    """Every parity case runs on both rollout kernels: the role-split one (the default at one
    workgroup per CU) and the pair kernel (the default at larger K), forced by MPPI_ROLES, which
    a context reads when it is created."""
    monkeypatch.setenv("MPPI_ROLES", "1" if request.param == "roles" else "0")
    return request.param


def _run_both(K, H, seed, st, proj="3d", step=0, nominal=None, scene=None, **pkw):
    Z, hw, cm = scene if scene is not None else hp.c3_scene()
    p = R.Params(K=K, H=H, seed=seed, **pkw)
    sc = hp.oracle_scene(Z, hw, cm)
    u1n, u2n = nominal if nominal is not None else (np.zeros(H, np.float32), np.zeros(H, np.float32))
    ref = R.mppi_step(p, sc, st, u1n, u2n, step, proj=proj)
    eng = hp.engine_for(K, H, Z, hw, cm, st, seed=seed, **pkw)
    if nominal is not None:
        eng.set_nominal(u1n, u2n)
    out = eng.step(proj, step)
    return ref, out, eng


def _assert_step(ref, out, eng):
    costs = eng.costs()
    assert np.array_equal(costs, ref["cost"]), hp.mismatch_report("cost", costs, ref["cost"])
    for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt")):
        assert hp.rel_err(out[a], ref[b]) <= TOL, hp.mismatch_report(a, out[a], ref[b])
    for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt"),
                 ("traj_sim", "traj_sim"), ("heading_sim", "hv_sim"), ("left_wheel_sim", "lw_sim"),
                 ("right_wheel_sim", "rw_sim")):
        assert np.array_equal(out[a], ref[b]), hp.mismatch_report(a, out[a], ref[b])


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("K,H", [(256, 20), (4096, 50)])
def test_step_parity_c1_c2(K, H, seed):
    st = hp.oracle_state()
    ref, out, eng = _run_both(K, H, seed, st)
    _assert_step(ref, out, eng)


def test_rollout_dump_bitexact():
    K, H = 300, 24     # ragged K (not a multiple of 256), even H
    st = hp.oracle_state(wl=0.3, wr=0.5)
    ref, out, eng = _run_both(K, H, 5, st, step=3)
    d = eng.dump()
    part = ref["parts"][0]
    for name, key in (("u1", "u1"), ("u2", "u2"), ("v", "v"), ("w", "w"), ("traj", "traj"), ("hv", "hv"),
                      ("lw", "lw"), ("rw", "rw")):
        assert np.array_equal(d[name], part[key]), hp.mismatch_report(name, d[name], part[key])
    _assert_step(ref, out, eng)


def test_odd_horizon_and_tiny_k():
    st = hp.oracle_state()
    for K, H in ((1, 7), (65, 9), (257, 3), (513, 1)):
        ref, out, eng = _run_both(K, H, 11, st)
        _assert_step(ref, out, eng)


@pytest.mark.parametrize("K,H,proj", [(256, 20, "3d"), (1000, 33, "3d"), (4096, 50, "3d"), (700, 24, "2d"),
                                      (513, 41, "3d"), (2048, 64, "2d")])
def test_rollout_dump_parity_shapes(K, H, proj):
    st = hp.oracle_state(wl=0.2, wr=0.1)
    ref, out, eng = _run_both(K, H, 8, st, proj=proj, step=2)
    _assert_step(ref, out, eng)
    d = eng.dump()
    part = ref["parts"][0]
    for name, key in (("u1", "u1"), ("u2", "u2"), ("v", "v"), ("w", "w"), ("traj", "traj"), ("hv", "hv"),
                      ("lw", "lw"), ("rw", "rw")):
        assert np.array_equal(d[name], part[key]), hp.mismatch_report(f"{K}x{H}:{name}", d[name], part[key])


def test_proj_2d_parity():
    st = hp.oracle_state()
    ref, out, eng = _run_both(512, 30, 4, st, proj="2d")
    _assert_step(ref, out, eng)
    d = eng.dump()
    assert np.array_equal(d["traj"], ref["parts"][0]["traj"])
    assert not d["lw"].any() and not d["rw"].any()


def test_goal_within_horizon_and_near_goal():
    # d <= horizon -> path-follow sum branch; d < 2 -> speed critic off
    st = hp.oracle_state(goal=(-57.0, -4.0))
    ref, out, eng = _run_both(512, 40, 6, st)
    _assert_step(ref, out, eng)
    st = hp.oracle_state(goal=(-59.0, -4.5))
    ref, out, eng = _run_both(512, 40, 6, st)
    _assert_step(ref, out, eng)


def test_collision_costs_and_nonzero_nominal():
    # start next to an obstacle cluster so rollouts cross costmap > 0.99
    Z, hw, cm = hp.c3_scene()
    ys, xs = np.nonzero(cm > 0.99)
    j, i = ys[len(ys) // 2], xs[len(xs) // 2]
    res_c = 2 * hw / cm.shape[0]
    x = -hw + (i + 0.5) * res_c - 2.0
    y = hw - (j + 0.5) * res_c
    st = hp.oracle_state(x=x, y=y, heading=(1.0, 0.2, 0.0), wl=0.4, wr=0.6, s1=0.4, s2=0.5)
    H = 48
    rng = np.random.RandomState(3)
    nom = (rng.uniform(-0.5, 0.8, H).astype(np.float32), rng.uniform(-0.5, 0.8, H).astype(np.float32))
    ref, out, eng = _run_both(2048, H, 9, st, step=17, nominal=nom)
    assert (ref["cost"] > 1e5).any(), "scene did not produce collisions"
    _assert_step(ref, out, eng)


@pytest.mark.parametrize("corner", [1.0, -1.0], ids=["upper", "lower"])
def test_map_edge_clamping(corner):
    # robot at a map corner heading out: cells outside the DEM/costmap are clamped (DEFINED
    # semantics); the optimal rollout's neighbourhood then holds repeated border cells
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(x=corner * (hw - 0.35), y=corner * (hw - 0.25), heading=(corner, corner, 0.0))
    ref, out, eng = _run_both(512, 40, 2, st)
    _assert_step(ref, out, eng)


def test_injected_controls():
    K, H = 700, 32
    st = hp.oracle_state()
    rng = np.random.RandomState(0)
    u1 = rng.uniform(-1, 1, (K, H)).astype(np.float32)
    u2 = rng.uniform(-1, 1, (K, H)).astype(np.float32)
    Z, hw, cm = hp.c3_scene()
    p = R.Params(K=K, H=H)
    ref = R.mppi_step(p, hp.oracle_scene(Z, hw, cm), st, np.zeros(H, np.float32), np.zeros(H, np.float32),
                      0, injected=(u1, u2))
    eng = hp.engine_for(K, H, Z, hw, cm, st)
    out = eng.step_injected(u1, u2)
    _assert_step(ref, out, eng)


def test_multi_step_closed_loop_nominal_chain():
    """Three consecutive steps: the engine's nominal-sequence hand-over equals the oracle's."""
    K, H = 1024, 30
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state()
    p = R.Params(K=K, H=H, seed=7)
    sc = hp.oracle_scene(Z, hw, cm)
    eng = hp.engine_for(K, H, Z, hw, cm, st, seed=7)
    u1n = np.zeros(H, np.float32)
    u2n = np.zeros(H, np.float32)
    for step in range(3):
        ref = R.mppi_step(p, sc, st, u1n, u2n, step)
        out = eng.step("3d", step)
        _assert_step(ref, out, eng)
        u1n, u2n = ref["u1_opt"], ref["u2_opt"]
        g1, g2 = eng.get_nominal()
        assert np.array_equal(g1, u1n) and np.array_equal(g2, u2n)
