"""CPU: pin the oracle (CPU restatement) against the reference's own numpy model and rocRAND.

Fixtures come from tests/golden/make_golden.py (reference debug.py imported in
the build container; rocRAND's Philox run on the host).  The reference computes
in float64, the restatement in float32 on the same float32 operands, so the
tolerances below are float32 rounding bounds.
"""
import os

import numpy as np
import pytest

from oracle import dmath
from oracle import mppi_ref as R

GOLD = os.path.join(os.path.dirname(__file__), "golden")
F32 = np.float32


@pytest.fixture(scope="module")
def prim():
    with np.load(os.path.join(GOLD, "ref_primitives.npz")) as f:
        return {k: f[k] for k in f.files}


def _q(q):
    q = q.astype(F32)
    return (q[:, 0, 0], q[:, 0, 1], q[:, 1, 0], q[:, 1, 1])


def test_normal_matches_debug(prim):
    """A5: projection_warp.py:129-151 == debug.py:200-216."""
    n = R.normal_on_grid(_q(prim["normal_q"]), prim["normal_res"].astype(F32))
    got = np.stack(n, axis=1).astype(np.float64)
    err = np.abs(got - prim["normal_out"])
    # cancellation in (q01-q00-q10+q11): error ~ ulp(|q|)/res on a unit vector
    tol = 8 * np.finfo(F32).eps * (1.0 + 6.0 / prim["normal_res"])[:, None]
    assert np.all(err <= tol), float(err.max())


def test_tangent_matches_debug(prim):
    """A6: projection_warp.py:168-190 == debug.py:218-232."""
    nv = tuple(prim["tangent_n"][:, i].astype(F32) for i in range(3))
    hv = tuple(prim["tangent_h"][:, i].astype(F32) for i in range(3))
    got = np.stack(R.heading_tangent(nv, hv), axis=1).astype(np.float64)
    assert np.max(np.abs(got - prim["tangent_out"])) < 2e-6


def test_rotation_matches_scipy_rotvec(prim):
    """A7: Rodrigues rotation (projection_warp.py:225-248) == scipy from_rotvec (debug.py:286-288)."""
    h = tuple(prim["rot_h"][:, i].astype(F32) for i in range(3))
    nv = tuple(prim["rot_n"][:, i].astype(F32) for i in range(3))
    x, y, v, w, dt = (prim[k].astype(F32) for k in ("rot_x", "rot_y", "rot_v", "rot_w", "rot_dt"))
    nx, ny = R.update_position(x, y, h, v, dt)
    nh = R.update_orientation(h, w, nv, dt)
    xy = np.stack([nx, ny], axis=1).astype(np.float64)
    assert np.max(np.abs(xy - prim["rot_out_xy"])) < 1e-5          # |x| <= 50: ulp 3.8e-6
    got = np.stack(nh, axis=1).astype(np.float64)
    assert np.max(np.abs(got - prim["rot_out_h"])) < 2e-6


def test_bilinear_matches_debug_positive_quadrant(prim):
    """A4 on x, y >= 0 where trunc == floor (projection_warp.py:70-100 vs debug.py:234-257)."""
    x, y, res = prim["bil_x"].astype(F32), prim["bil_y"].astype(F32), prim["bil_res"].astype(F32)
    got = R.bilinear(x, y, _q(prim["bil_q"]), res).astype(np.float64)
    # fraction of x/res (up to 1600) carries ulp(1600)=1.2e-4 in float32; heights <= 3
    err = np.abs(got - prim["bil_out"])
    tol = 4 * 3.0 * np.finfo(F32).eps * np.maximum(prim["bil_x"], prim["bil_y"]) / prim["bil_res"] + 1e-6
    assert np.all(err <= tol), float(err.max())


def test_bilinear_trunc_quirk_negative_coords():
    """A4 for x<0: Warp's int() truncates, so the fraction is negative."""
    q = (F32(1.0), F32(2.0), F32(3.0), F32(5.0))
    x, y, res = F32(-0.25), F32(-0.25), F32(0.1)
    h = R.bilinear(np.array([x]), np.array([y]), q, res)[0]
    xn, yn = np.float64(x) / np.float64(res), np.float64(y) / np.float64(res)
    x2, y2 = xn - np.trunc(xn), yn - np.trunc(yn)          # -0.5, -0.5
    want = (1 - x2) * (1 - y2) * 1.0 + x2 * (1 - y2) * 3.0 + (1 - x2) * y2 * 2.0 + x2 * y2 * 5.0
    assert abs(float(h) - want) < 1e-5
    assert abs(want - 1.0) > 0.5     # floor would give a value inside the cell; trunc extrapolates


def test_philox_matches_rocrand():
    rows = np.loadtxt(os.path.join(GOLD, "philox_rocrand.txt"), dtype=np.uint64, comments="#")
    assert rows.shape == (100, 7)
    for s, k, n, *r in rows:
        s, k, n = int(s), int(k), int(n)
        got = dmath.philox4x32_10(n & 0xFFFFFFFF, n >> 32, k & 0xFFFFFFFF, k >> 32, s & 0xFFFFFFFF, s >> 32)
        assert [int(g) for g in got] == [int(v) for v in r], (s, k, n)


def test_philox_published_kat():
    """Random123 kat_vectors for philox4x32_10 (counter=key=0, all-ones, pi digits)."""
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
        ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
        ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
         (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
    ]
    for c, k, want in cases:
        got = dmath.philox4x32_10(*c, *k)
        assert [int(g) for g in got] == list(want)


def test_dmath_accuracy():
    """Cephes-style f32 transcendentals stay within a few ulp of float64 libm."""
    x = np.linspace(1e-7, 1.0, 200001, dtype=F32)
    rel = np.abs(dmath.dm_logf(x).astype(np.float64) - np.log(x.astype(np.float64)))
    assert np.max(rel / np.maximum(np.abs(np.log(x.astype(np.float64))), 1e-30)) < 4e-7 or np.max(rel) < 3e-7
    e = np.linspace(-80.0, 0.0, 200001, dtype=F32)
    ex = np.exp(e.astype(np.float64))
    assert np.max(np.abs(dmath.dm_expf(e) - ex) / ex) < 4e-7
    a = np.linspace(-8.0, 8.0, 200001, dtype=F32)
    s, c = dmath.dm_sincosf(a)
    assert np.max(np.abs(s - np.sin(a.astype(np.float64)))) < 3e-7
    assert np.max(np.abs(c - np.cos(a.astype(np.float64)))) < 3e-7


def test_box_muller_moments():
    k = np.arange(1 << 16, dtype=np.int64)
    z = np.concatenate(dmath.noise_block(42, 3, k)).astype(np.float64)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    assert np.all(np.isfinite(z))


@pytest.fixture(scope="module")
def steps():
    with np.load(os.path.join(GOLD, "step_small.npz")) as f:
        return {k: f[k] for k in f.files}


@pytest.mark.parametrize("name", ["far3d", "near3d", "twod", "ragged", "injected"])
def test_oracle_step_regression(steps, name):
    """The restatement still reproduces its frozen whole-step vectors bit for bit."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    out = mg.run_step_case(name, steps["Z"], float(steps["hw"]), steps["cm"])
    for key, val in out.items():
        np.testing.assert_array_equal(val, steps[f"{name}/{key}"], err_msg=f"{name}/{key}")


def test_sincos_small_angle_path_equals_general():
    """dm_sincosf_small (the rollout's sin / cos of w dt when max|w| dt < 0.78, no range reduction)
    gives dm_sincosf's bits on every float32 in [-0.78, 0.78] sampled densely (all floats in
    [2^-12, 2^-11) and [0.75, 0.78], 4 M random ones, zeros, the bound) — both signs."""
    rng = np.random.default_rng(5)
    lo = np.arange(np.float32(2.0 ** -12).view(np.uint32), np.float32(2.0 ** -11).view(np.uint32), dtype=np.uint32)
    hi = np.arange(np.float32(0.75).view(np.uint32), np.float32(0.78).view(np.uint32), dtype=np.uint32)
    x = np.concatenate([lo.view(F32), hi.view(F32), rng.uniform(0, 0.78, 4_000_000).astype(F32),
                        np.array([0.0, 1e-30, 0.78, 0.045], F32)])
    x = np.concatenate([x, -x])
    assert np.all(np.abs(x) * dmath.FOPI < F32(1.0))
    s0, c0 = dmath.dm_sincosf(x)
    s1, c1 = dmath.dm_sincosf_small(x)
    assert np.array_equal(s0.view(np.uint32), s1.view(np.uint32))
    assert np.array_equal(c0.view(np.uint32), c1.view(np.uint32))
