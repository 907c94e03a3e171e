"""GPU: config C5 (BASELINE.json configs[4]) — K=262144, H=128 on an 8192^2 DEM @0.025 m.

The same bar as C1-C3: costs bit-exact with the numpy restatement (oracle/), emitted controls
within 1e-5 relative.  The sampled check runs the oracle on a 2048-trajectory slice at a
global offset (Philox is keyed by the global trajectory index, so the slice's samples are the
full run's); the full-size check runs the whole C5 step on both sides (~20-40 s of numpy).
"""
import functools

import numpy as np
import pytest

import helpers as hp
from oracle import mppi_ref as R

pytestmark = pytest.mark.gpu

TOL = 1e-5
K5, H5 = 262144, 128
START5 = (0.0, 0.0)
GOAL5 = (80.0, 20.0)


@functools.lru_cache(maxsize=1)
def _scene():
    from mppi_amd import scene
    return scene.scene_c5()


def _state(**kw):
    return hp.oracle_state(x=START5[0], y=START5[1], goal=GOAL5, **kw)


def _assert_controls(out, ref):
    for a, b in (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt")):
        assert hp.rel_err(out[a], ref[b]) <= TOL, hp.mismatch_report(a, out[a], ref[b])
        assert np.array_equal(out[a], ref[b]), hp.mismatch_report(a, out[a], ref[b])
    for a, b in (("traj_sim", "traj_sim"), ("heading_sim", "hv_sim"), ("left_wheel_sim", "lw_sim"),
                 ("right_wheel_sim", "rw_sim")):
        assert np.array_equal(out[a], ref[b]), hp.mismatch_report(a, out[a], ref[b])


def test_c5_slice_bitexact():
    """2048 trajectories at global offset 131072 of the C5 sample set, H=128, 8192^2 DEM."""
    Z, hw, cm = _scene()
    st = _state(wl=0.2, wr=0.3)
    K, k0 = 2048, 131072
    p = R.Params(K=K, H=H5, seed=42)
    sc = R.Scene(Z, hw, cm)
    rec, part = R.shard_record(p, sc, st, np.zeros(H5, np.float32), np.zeros(H5, np.float32), 4, k0, K)
    ref = R.finish(p, sc, st, rec)
    ref["cost"] = part["cost"]
    eng = hp.engine_for(K, H5, Z, hw, cm, st, seed=42, k_offset=k0)
    out = eng.step("3d", 4)
    assert np.array_equal(eng.costs(), ref["cost"]), hp.mismatch_report("cost", eng.costs(), ref["cost"])
    _assert_controls(out, ref)
    d = eng.dump()
    for name in ("traj", "hv", "lw", "rw"):
        assert np.array_equal(d[name], part[name]), hp.mismatch_report(name, d[name], part[name])
    eng.close()


def test_c5_full_size_step():
    """The whole C5 step (262144 trajectories) against the oracle's: costs and emitted controls."""
    Z, hw, cm = _scene()
    st = _state()
    p = R.Params(K=K5, H=H5, seed=42)
    ref = R.mppi_step(p, R.Scene(Z, hw, cm), st, np.zeros(H5, np.float32), np.zeros(H5, np.float32), 0)
    eng = hp.engine_for(K5, H5, Z, hw, cm, st, seed=42)
    out = eng.step("3d", 0)
    costs = eng.costs()
    assert np.array_equal(costs, ref["cost"]), hp.mismatch_report("cost", costs, ref["cost"])
    _assert_controls(out, ref)
    eng.close()
