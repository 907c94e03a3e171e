"""GPU: the HIP obstacle-costmap builder (csrc/mppi_costmap.hip) vs oracle/costmap_ref.py.

Surface.create_obstacles_costmap (MPPI_isaac.py:361-378) with both distance metrics: "chamfer",
the reference's cv2.distanceTransform(DIST_L2, 5) restated from OpenCV's published 5x5 chamfer
(parity unpinned: no cv2 here), and "exact", the exact EDT.  Raster and the
fixed-point / squared distances are integer work and must match exactly; the normalise + power
are expected bit-exact too (both sides round the power correctly), so the test asserts equality
and reports any cell that differs.
"""
import numpy as np
import pytest

import helpers as hp
from oracle import costmap_ref as CR

pytestmark = pytest.mark.gpu


def _rocks(n, extent, seed, rmax=0.8):
    rng = np.random.RandomState(seed)
    return [[rng.uniform(-extent, extent), rng.uniform(-extent, extent), rng.uniform(0.0, rmax)] for _ in range(n)]


@pytest.fixture(scope="module")
def builder():
    from mppi_amd import _lib
    b = _lib.CostmapBuilder(0)
    yield b
    b.close()


CASES = {
    # name: (obstacles, origin, size, half_width, r_robot, power)
    "tiny": (_rocks(3, 2.0, 0), (0.0, 0.0), 2, 3.0, 1.2, 20),
    "odd": (_rocks(12, 8.0, 1), (0.4, -0.7), 65, 10.0, 1.2, 20),
    "ref_875": (_rocks(600, 80.0, 2), (3.5, -12.25), 875, 87.5, 1.2, 20),     # 7000^2 HR DEM / 8
    "c5_1024": (_rocks(2000, 95.0, 3), (0.0, 0.0), 1024, 102.4, 1.2, 20),
    "power10": (_rocks(750, 50.0, 99, 0.4), (0.0, 0.0), 750, 75.0, 0.3, 10),
    "sparse": (_rocks(2, 30.0, 4), (0.0, 0.0), 500, 40.0, 1.2, 20),            # long empty columns / rows
    "outside": ([[500.0, 500.0, 1.0], [1.0, 2.0, 0.5]], (0.0, 0.0), 128, 12.8, 1.2, 20),
    "none": ([], (0.0, 0.0), 96, 9.6, 1.2, 20),
    "all": ([[0.0, 0.0, 500.0]], (0.0, 0.0), 64, 6.4, 1.2, 20),
    "power0": (_rocks(10, 5.0, 5), (0.0, 0.0), 40, 6.0, 1.2, 0),
    # one small disc in a corner of a 1024^2 map: the longest lines of every scan direction
    "corner_1024": ([[-101.0, -101.0, 0.1]], (0.0, 0.0), 1024, 102.4, 0.05, 20),
    "rect_edge": ([[12.7, -3.0, 0.2], [-12.0, 12.6, 0.3]], (0.0, 0.0), 255, 12.8, 0.1, 20),
}


# "chamfer" runs the 16 line scans, "chamfer_raster" the row-serial raster passes (same map)
ORACLE = {"chamfer": CR.create_obstacles_costmap_cv, "chamfer_raster": CR.create_obstacles_costmap_cv,
          "exact": CR.create_obstacles_costmap}


@pytest.mark.parametrize("metric", list(ORACLE))
@pytest.mark.parametrize("name", list(CASES))
def test_builder_matches_oracle(builder, name, metric):
    obs, origin, size, hw, rr, power = CASES[name]
    want = ORACLE[metric](obs, origin, size, hw, rr, power)
    got = builder.build(obs, origin, size, hw, rr, power, metric=metric)
    assert got.shape == want.shape and got.dtype == np.float32
    assert np.array_equal(got, want), hp.mismatch_report(name, got, want)


def test_engine_build_costmap_equals_upload():
    """mppi_build_costmap writes the context's costmap in place: a step afterwards is bitwise the
    step after uploading the oracle's map with set_costmap (the reference's assign)."""
    Z, hw, _ = hp.c3_scene()
    st = hp.oracle_state()
    obs = _rocks(750, 50.0, 99, 0.4)
    want = CR.create_obstacles_costmap_cv(obs, (1.0, -2.0), 187, hw, 1.2, 20)   # grid 1500 / 8
    e1 = hp.engine_for(1024, 40, Z, hw, want, st)
    out1 = e1.step("3d", 0)
    e2 = hp.engine_for(1024, 40, Z, hw, np.zeros((4, 4), np.float32), st)
    got = e2.build_costmap(obs, (1.0, -2.0), 187, hw, 1.2, 20)
    assert np.array_equal(got, want), hp.mismatch_report("costmap", got, want)
    out2 = e2.step("3d", 0)
    assert np.array_equal(e1.costs(), e2.costs())
    for k in out1:
        assert np.array_equal(out1[k], out2[k]), k
    e1.close()
    e2.close()


def test_surface_manual_costmap_on_gpu():
    """Surface("manual", ..., "manual", ...) builds its costmap with the HIP builder (MPPI_isaac.py:287-291)."""
    from mppi_amd import scene
    from mppi_amd.controller import Surface
    obstacles = [[3.0, -2.0, 0.8], [-4.0, 5.0, 1.2]]
    s = Surface("manual", None, "manual", None, 160, 8.0, (0.0, 0.0), scene.BUMPS_9[:2], 1.2, obstacles)
    assert s.costmap.shape == (20, 20)
    want = CR.create_obstacles_costmap_cv(obstacles, (0.0, 0.0), 20, 8.0, 1.2, 20)
    assert np.array_equal(s.costmap, want)


def test_bad_arguments_raise(builder):
    with pytest.raises(RuntimeError):
        builder.build([[0, 0, 1]], (0, 0), 1, 5.0, 1.2)
    with pytest.raises(RuntimeError):
        builder.build([[0, 0, 1]], (0, 0), 9000, 5.0, 1.2)
    with pytest.raises(ValueError):
        builder.build([[0, 0, 1]], (0, 0), 16, 5.0, 1.2, metric="l1")
