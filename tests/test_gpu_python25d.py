"""GPU: the HIP reference-integrator mode "python25d" (csrc/mppi_python25d.hip) reproduces whole
trajectories of the reference's numpy integrator debug.generate_trajectory_25D (debug.py:312-364),
frozen in tests/golden/python25d.npz, and the oracle restatement at a larger batch."""
import os

import numpy as np
import pytest

from oracle import python25d_ref as P

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "python25d.npz")
ATOL = 1e-10   # float64 end to end; ocml vs libm sin/cos may differ in the last bit


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD) as f:
        return {k: f[k] for k in f.files}


@pytest.fixture(scope="module")
def engine(gold):
    from mppi_amd import _lib
    eng = _lib.Engine(_lib.make_params(256, 8), 0)
    eng.set_dem(gold["Z"], float(gold["hw"]))
    yield eng
    eng.close()


@pytest.mark.parametrize("case", ["demo", "escape"])
def test_gpu_matches_reference_trajectories(gold, engine, case):
    g = lambda k: gold[f"{case}/{k}"]  # noqa: E731
    traj, valid = engine.rollout_python25d(g("x0"), g("y0"), g("heading"), g("v"), g("w"), float(g("dt")),
                                           float(gold["hw"]), float(gold["res"]))
    assert np.array_equal(valid, g("valid"))
    err = np.abs(traj[valid] - g("traj")[valid]).max()
    assert err <= ATOL, err


def test_gpu_matches_oracle_batch(gold, engine):
    rng = np.random.default_rng(3)
    K, H, dt = 4096, 120, 0.05
    x0 = rng.uniform(-16, 16, K)
    y0 = rng.uniform(-16, 16, K)
    hd = np.stack([rng.normal(size=K), rng.normal(size=K), rng.normal(size=K) * 0.1], 1)
    v = rng.uniform(0.0, 2.5, (K, H))
    w = rng.uniform(-1.0, 1.0, (K, H))
    w[:8] = 0.0                                  # straight lines: rotvec Taylor branch at angle 0
    w[8:16] = 1e-3 / dt * rng.uniform(0.5, 1.0, (8, H))   # around the 1e-3 rad Taylor threshold
    Z = gold["Z"].astype(np.float64)
    want, wvalid = P.generate_trajectories_25d(x0, y0, hd, v, w, dt, Z, float(gold["hw"]), float(gold["res"]))
    got, gvalid = engine.rollout_python25d(x0, y0, hd, v, w, dt, float(gold["hw"]), float(gold["res"]))
    assert np.array_equal(gvalid, wvalid)
    assert (~wvalid).any() and wvalid.any()
    assert np.abs(got - want).max() <= ATOL
