"""GPU: the headline config C3 (K=65536, H=100, BASELINE.json configs[1]) and C4's K=1,048,576
against the numpy restatement (oracle/) at FULL size, through the C-ABI.

Bar (north_star): emitted controls within 1e-5 relative; costs, controls and the optimal rollout
are expected bit-exact (every float op is defined identically on both sides) and asserted so.
Reference step: thesis_master/warp_implementation/MPPI_isaac.py:505-720.

C4 is 1,048,576 trajectories on ONE GPU here (the 8-GPU split is the same records, §8(e)); the
oracle computes it as 16 aligned 65,536-trajectory chunks whose roots combine with the same binary
tree (every chunk is a power-of-two number of 256-trajectory leaves, so the chunk roots are
exactly the subtrees of the 4096-leaf tree).
"""
import numpy as np
import pytest

import helpers as hp
from oracle import mppi_ref as R

pytestmark = pytest.mark.gpu

TOL = 1e-5
K3, H3 = 65536, 100
K4 = 1048576


def _zeros(H):
    return np.zeros(H, np.float32), np.zeros(H, np.float32)


def _assert_reference_f32(out, ref, p, st, T_tol=TOL):
    """The emitted controls against the reference's OWN float32 update (critics_warp.py:338-376,
    9 atomic orders; tests/test_reference_update.py): per element within 1e-5."""
    part = ref["parts"][0]
    worst = 0.0
    for o in R.reference_emitted_f32(p, st, part["cost"], part["u1"], part["u2"]):
        for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt")):
            worst = max(worst, hp.rel_err(out[a], o[b]))
    print(f"reference-f32 update: worst per-element rel err {worst:.3e}")
    assert worst <= T_tol, worst


def _assert_outputs(out, ref, costs):
    assert np.array_equal(costs, ref["cost"]), hp.mismatch_report("cost", costs, ref["cost"])
    for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt")):
        assert hp.rel_err(out[a], ref[b]) <= TOL, hp.mismatch_report(a, out[a], ref[b])
    for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt"),
                 ("traj_sim", "traj_sim"), ("heading_sim", "hv_sim"), ("left_wheel_sim", "lw_sim"),
                 ("right_wheel_sim", "rw_sim")):
        assert np.array_equal(out[a], ref[b]), hp.mismatch_report(a, out[a], ref[b])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_c3_full_step(seed):
    """One full C3 step, 65,536 trajectories x 100 steps, robot at the bench start pose."""
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(wl=0.1 * seed, wr=0.15 * seed)
    p = R.Params(K=K3, H=H3, seed=seed)
    ref = R.mppi_step(p, hp.oracle_scene(Z, hw, cm), st, *_zeros(H3), 0)
    eng = hp.engine_for(K3, H3, Z, hw, cm, st, seed=seed)
    out = eng.step("3d", 0)
    _assert_outputs(out, ref, eng.costs())
    _assert_reference_f32(out, ref, p, st)
    eng.close()


@pytest.mark.parametrize("T", [3000.0, 1e5])
def test_c3_reference_f32_raised_temperature(T):
    """C3 with a raised temperature (~1 000 / ~15 500 effective samples, where the reference's
    float32 summation order matters): the engine is bit-exact with the oracle, its u_opt is the
    exact weighted mean of the reference's float32 weights (< 1e-7), and its distance to the
    reference's 9 float32 orderings (whole-vector metric) is reported; T = 3000 must be within
    1e-5, T = 1e5 within the reference's own float32 drift of 5e-5; per element, the engine lies
    within ENVELOPE_TOL (2e-5) of the orderings' envelope."""
    from test_reference_update import ENVELOPE_TOL, exact_mean, glob_err, outside_envelope
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(wl=0.1, wr=0.15)
    p = R.Params(K=K3, H=H3, seed=1, temperature=T)
    ref = R.mppi_step(p, hp.oracle_scene(Z, hw, cm), st, *_zeros(H3), 0)
    eng = hp.engine_for(K3, H3, Z, hw, cm, st, seed=1, temperature=T)
    out = eng.step("3d", 0)
    _assert_outputs(out, ref, eng.costs())
    part = ref["parts"][0]
    for k, u in (("u1_opt", part["u1"]), ("u2_opt", part["u2"])):
        assert glob_err(out[k], exact_mean(part["cost"], u, T)) < 1e-7
    worst = 0.0
    for o in R.reference_emitted_f32(p, st, part["cost"], part["u1"], part["u2"]):
        for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt")):
            worst = max(worst, glob_err(out[a], o[b]))
    outs = R.reference_emitted_f32(p, st, part["cost"], part["u1"], part["u2"])
    env = max(outside_envelope(out[a], [o[b] for o in outs])
              for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt")))
    print(f"T={T}: reference-f32 update, worst whole-vector rel err {worst:.3e}, per element outside the "
          f"orderings' envelope {env:.3e}")
    assert worst <= (TOL if T <= 3000.0 else 5e-5), worst
    assert env <= ENVELOPE_TOL, env  # (measured on the oracle: 6.2e-6 at T = 3000, 1.3e-5 at T = 1e5)
    eng.close()


def test_c3_closed_loop_three_steps():
    """Three consecutive C3 steps: each step samples around the previous step's u_opt (the
    engine keeps it on the device, the oracle is handed it), step counters 0, 1, 2."""
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(wl=0.2, wr=0.25)
    p = R.Params(K=K3, H=H3, seed=42)
    sc = hp.oracle_scene(Z, hw, cm)
    eng = hp.engine_for(K3, H3, Z, hw, cm, st, seed=42)
    u1, u2 = _zeros(H3)
    for n in range(3):
        ref = R.mppi_step(p, sc, st, u1, u2, n)
        out = eng.step("3d", n)
        _assert_outputs(out, ref, eng.costs())
        u1, u2 = ref["u1_opt"], ref["u2_opt"]
    eng.close()


def test_c4_full_size_step():
    """K=1,048,576, H=100 (BASELINE.json configs[3]) in one context: all costs and the emitted
    controls against the oracle's chunked evaluation."""
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(wl=0.05, wr=0.1)
    p = R.Params(K=K4, H=H3, seed=7)
    sc = hp.oracle_scene(Z, hw, cm)
    chunk = 65536
    recs, costs = [], []
    for b in range(0, K4, chunk):
        rec, part = R.shard_record(p, sc, st, *_zeros(H3), 0, b, chunk)
        recs.append(rec)
        costs.append(part["cost"])
        del part
    ref = R.finish(p, sc, st, R.tree_reduce(np.stack(recs), p.temperature))
    ref["cost"] = np.concatenate(costs)
    eng = hp.engine_for(K4, H3, Z, hw, cm, st, seed=7)
    out = eng.step("3d", 0)
    _assert_outputs(out, ref, eng.costs())
    info = eng.launch_info()   # 4096 records at H=100: the record-tree finish (column split does not fit)
    assert info["finish_kind"] == 0 and info["finish_records"] == 4096 and info["blocks"] == 4096
    eng.close()


def test_c4_slice_high_offset():
    """A 4096-trajectory slice at global offset 1,044,480 (the last 4096 of C4's sample set):
    Philox keyed by the global index gives the full run's samples; rollouts bit-exact too."""
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state(wl=0.3, wr=0.2)
    K, k0 = 4096, K4 - 4096
    p = R.Params(K=K, H=H3, seed=11)
    sc = hp.oracle_scene(Z, hw, cm)
    rec, part = R.shard_record(p, sc, st, *_zeros(H3), 2, k0, K)
    ref = R.finish(p, sc, st, rec)
    ref["cost"] = part["cost"]
    eng = hp.engine_for(K, H3, Z, hw, cm, st, seed=11, k_offset=k0)
    out = eng.step("3d", 2)
    _assert_outputs(out, ref, eng.costs())
    d = eng.dump()
    for name in ("traj", "hv", "lw", "rw"):
        assert np.array_equal(d[name], part[name]), hp.mismatch_report(name, d[name], part[name])
    eng.close()
