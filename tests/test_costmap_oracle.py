"""CPU: the obstacle-costmap restatement (oracle/costmap_ref.py, MPPI_isaac.py:361-378).

Pins the exact-EDT call against an exhaustive search, the vectorised 5x5 chamfer (OpenCV's
distanceTransform_5x5, the reference's cv2.distanceTransform(DIST_L2, 5)) against its literal
per-pixel loop, and the raster against the reference's frame convention (x_local = y_global - y0
marks a COLUMN coordinate, y_local = x_global - x0 a ROW coordinate of
meshgrid(linspace(-hw, hw, size))).  cv2 itself is absent: the chamfer restatement is "parity
unpinned" against it.
"""
import numpy as np
import pytest

from oracle import costmap_ref as CR


def _rocks(n, extent, seed):
    rng = np.random.RandomState(seed)
    return [[rng.uniform(-extent, extent), rng.uniform(-extent, extent), rng.uniform(0.0, 0.8)] for _ in range(n)]


@pytest.mark.parametrize("size,n,seed", [(48, 6, 0), (65, 15, 1), (80, 40, 2)])
def test_edt_matches_bruteforce(size, n, seed):
    occ = CR.raster(_rocks(n, 9.0, seed), (0.4, -0.7), size, 10.0, 1.2)
    assert occ.any() and not occ.all()
    assert np.array_equal(CR.edt(occ), CR.edt_bruteforce(occ))


def test_raster_frame_swap():
    # one small rock at global (x, y) = (2, -3), origin (0, 0): its disc is centred on
    # X = y_global = -3 (column), Y = x_global = 2 (row)
    size, hw = 101, 10.0
    occ = CR.raster([[2.0, -3.0, 0.0]], (0.0, 0.0), size, hw, 0.05)   # total radius 0.15 < cell 0.2
    js, is_ = np.nonzero(occ)
    x = np.linspace(-hw, hw, size)
    assert len(js) == 1 and x[is_[0]] == pytest.approx(-3.0) and x[js[0]] == pytest.approx(2.0)


def test_edge_cases():
    size = 32
    assert np.array_equal(CR.create_obstacles_costmap([], (0, 0), size, 5.0, 1.2), np.ones((size, size), np.float32))
    full = CR.create_obstacles_costmap([[0.0, 0.0, 100.0]], (0, 0), size, 5.0, 1.2)
    assert np.array_equal(full, np.ones((size, size), np.float32))
    cm = CR.create_obstacles_costmap(_rocks(5, 4.0, 3), (0, 0), size, 5.0, 0.3)
    assert cm.dtype == np.float32 and cm.max() == 1.0 and cm.min() == 0.0


@pytest.mark.parametrize("shape,p,seed", [((23, 31), 0.1, 0), ((40, 17), 0.01, 1), ((9, 64), 0.3, 2),
                                           ((33, 33), 0.0, 3), ((12, 12), 1.0, 4), ((1, 50), 0.05, 5)])
def test_chamfer_vectorised_matches_per_pixel_loop(shape, p, seed):
    occ = np.random.RandomState(seed).rand(*shape) < p
    assert np.array_equal(CR.chamfer_l2_5x5(occ), CR.chamfer_l2_5x5_loops(occ))


def test_chamfer_known_distances():
    """One obstacle pixel: the mask-5 metric {1, 1.4, 2.1969} in 16.16 fixed point along the axes,
    the diagonal and the knight's move."""
    occ = np.zeros((9, 9), bool)
    occ[4, 4] = True
    d = CR.chamfer_l2_5x5(occ)
    fx = lambda t: np.float32(np.float32(t) * np.float32(1 / 65536))
    assert d[4, 4] == 0
    assert d[4, 7] == fx(3 * 65536) and d[1, 4] == fx(3 * 65536)
    assert d[6, 6] == fx(2 * 91750)
    assert d[5, 6] == fx(143976) and d[2, 3] == fx(143976)


def test_chamfer_costmap_edges():
    size = 32
    full = CR.create_obstacles_costmap_cv([[0.0, 0.0, 100.0]], (0, 0), size, 5.0, 1.2)
    assert np.array_equal(full, np.ones((size, size), np.float32))   # min == max: scale 0
    cm = CR.create_obstacles_costmap_cv(_rocks(5, 4.0, 3), (0, 0), size, 5.0, 0.3)
    assert cm.dtype == np.float32 and cm.max() == 1.0 and cm.min() == 0.0


def test_fmaf32_single_rounding():
    """The oracle's float32 fma (cv::normalize's convertTo, v_fma) rounds once: against exact
    rational arithmetic on random operands and on constructed halfway cases."""
    from fractions import Fraction
    rng = np.random.default_rng(3)
    x = rng.random(4000).astype(np.float32)
    a = np.float32(rng.random() * 3 + 0.1)
    b = np.float32(-rng.random())
    # operands whose float64 sum lands exactly on a float32 midpoint with a non-zero error term
    x = np.concatenate([x, np.float32([1.0 + 2.0 ** -23, 1.5, 3.0])])
    got = CR.fmaf32(x, a, b)
    for xi, gi in zip(x, got):
        exact = Fraction(float(xi)) * Fraction(float(a)) + Fraction(float(b))
        lo = np.float32(float(exact))
        cands = [lo, np.nextafter(lo, np.float32(np.inf)), np.nextafter(lo, np.float32(-np.inf))]
        best = min(cands, key=lambda c: (abs(Fraction(float(c)) - exact), int(np.float32(c).view(np.uint32)) & 1))
        assert gi == best, (xi, gi, best)
    # midpoint construction: x * a + b = m + tiny where m is a float32 midpoint
    m = Fraction(1) + Fraction(1, 2 ** 24)          # halfway between 1 and 1 + 2^-23
    got = CR.fmaf32(np.float32([1.0]), np.float32(1.0), np.float32(2.0 ** -24))
    assert got[0] == np.float32(1.0)                # tie -> even (e == 0)
    assert m > 1


def test_cv_normalize_float32_path():
    """cv::normalize(NORM_MINMAX) for CV_32F: float scale / shift and a float32 fma."""
    d = np.float32([[0.5, 2.0], [7.25, 3.0]])
    out = CR.cv_normalize_minmax(d)
    scale = np.float32(1.0 / (7.25 - 0.5))
    shift = np.float32(0.0) - np.float32(0.5 * float(scale))
    exp = CR.fmaf32(d, scale, shift)
    np.testing.assert_array_equal(out, exp)
    assert out.dtype == np.float32 and out.min() == 0.0
    np.testing.assert_array_equal(CR.cv_normalize_minmax(np.full((3, 3), 2.0, np.float32)), np.zeros((3, 3), np.float32))


@pytest.mark.parametrize("shape,p,seed", [((1, 1), 1.0, 0), ((2, 9), 0.2, 1), ((37, 23), 0.01, 2),
                                          ((64, 64), 0.002, 3), ((97, 130), 0.05, 4), ((130, 97), 0.3, 5)])
def test_chamfer_line_scans_match_raster_passes(shape, p, seed):
    """The HIP builder's formulation (16 line scans) gives the raster passes' map bit for bit."""
    occ = np.random.default_rng(seed).random(shape) < p
    occ.flat[seed % occ.size] = True
    assert np.array_equal(CR.chamfer_l2_5x5_lines(occ).view(np.uint32), CR.chamfer_l2_5x5(occ).view(np.uint32))


@pytest.mark.parametrize("cell", [(0, 0), (0, 79), (59, 0), (59, 79), (30, 41)])
def test_chamfer_line_scans_single_cell(cell):
    """One obstacle cell: the longest paths of every sector, from every corner."""
    occ = np.zeros((60, 80), bool)
    occ[cell] = True
    assert np.array_equal(CR.chamfer_l2_5x5_lines(occ).view(np.uint32), CR.chamfer_l2_5x5(occ).view(np.uint32))
    assert CR.chamfer_l2_5x5_lines(np.zeros((5, 5), bool)) is None
