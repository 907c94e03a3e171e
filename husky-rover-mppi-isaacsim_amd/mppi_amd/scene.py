"""Synthetic scene recipes (the reference's .npy scene blobs are not in the repo).

SURVEY.md §0.5 / §8(d): ``costmap_750_*.npy`` and ``test_nathan.npy`` are
missing (.MISSING_LARGE_BLOBS), so every scene is regenerated from the
reference's own recipes:

* DEM craters: ``Surface.create_surface`` (thesis_master/warp_implementation/
  MPPI_isaac.py:307-356) with the 9-crater list of MPPI_OO_current.py:730-740,
  on the 1500^2 @ 0.1 m grid of MPPI_OO_current.py:209-213.
* Costmap: 750 random discs (MPPI_OO_current.py:721-725, RandomState(99)),
  inflated by robot radius + 0.2 (MPPI_OO_current.py:293), Euclidean distance
  transform, min-max normalise, ``(1 - d)**10`` (create_costmap.py:15-28).
  cv2.distanceTransform(DIST_L2, 5) is not available; scipy's exact EDT is used
  instead (parity of the costmap *builder* is unpinned; the costmap is an input
  of the hot path).

Host-side scene construction only: this is not on the MPPI step path.
"""
from __future__ import annotations

import numpy as np

# MPPI_OO_current.py:730-740 (commented scene block)
BUMPS_9 = [
    ((-2.7, -19.0), 3.4, 12.23),
    ((-0.57, -0.05), 4.39, 11.52),
    ((-48.56, 12.78), 3.6, 12.4),
    ((-27.89, 38.56), 4.0, 12.7),
    ((-50.12, 19.34), 3.7, 13.0),
    ((20.45, -48.78), 4.4, 12.9),
    ((-20.67, -40.12), 4.2, 12.9),
    ((42.78, 21.56), 4.5, 12.7),
    ((-36.12, -33.34), 3.9, 13.0),
]


def crater_dem(grid_size, half_width, bumps=BUMPS_9, scale=1.0):
    """Surface.create_surface (MPPI_isaac.py:307-356): crater = rim gaussian minus bowl gaussian."""
    x = np.linspace(-half_width, half_width, grid_size)
    X, Y = np.meshgrid(x, x)
    Z = np.zeros_like(X)
    for (cx, cy), h, w in bumps:
        cx, cy, w = cx * scale, cy * scale, w * scale
        r2 = (X - cx) ** 2 + (Y - cy) ** 2
        Z += (h - 0.5) * np.exp(-r2 / (2 * w ** 2))
        Z -= (h + 0.5) * np.exp(-r2 / (2 * (w / 2) ** 2))
    return Z.astype(np.float32)


def random_obstacles(n=750, seed=99, extent=50.0, r_max=0.4):
    """MPPI_OO_current.py:721-725: [x, y, r] with RandomState(seed)."""
    rng = np.random.RandomState(seed)
    return [[rng.uniform(-extent, extent), rng.uniform(-extent, extent), rng.uniform(0.0, r_max)]
            for _ in range(n)]


def edt_costmap(occupied, power=10):
    """create_costmap.py:15-28: distance to nearest obstacle -> min-max normalise -> (1-d)**power."""
    from scipy.ndimage import distance_transform_edt
    d = distance_transform_edt(~occupied).astype(np.float64)
    lo, hi = d.min(), d.max()
    dn = (d - lo) / (hi - lo) if hi > lo else np.zeros_like(d)
    return ((1.0 - dn) ** power).astype(np.float32)


def disc_costmap(size, half_width, obstacles, inflate=0.5, power=10):
    """Binary disc raster (MPPI_OO_current.py:291-296: r + r_robot(0.3) + 0.2) -> edt_costmap."""
    x = np.linspace(-half_width, half_width, size)
    X, Y = np.meshgrid(x, x)
    occ = np.zeros((size, size), bool)
    for ox, oy, r in obstacles:
        rr = r + inflate
        # bounding box only
        i0 = max(0, int((ox - rr + half_width) / (2 * half_width) * (size - 1)) - 1)
        i1 = min(size, int((ox + rr + half_width) / (2 * half_width) * (size - 1)) + 2)
        j0 = max(0, int((oy - rr + half_width) / (2 * half_width) * (size - 1)) - 1)
        j1 = min(size, int((oy + rr + half_width) / (2 * half_width) * (size - 1)) + 2)
        sub = (X[j0:j1, i0:i1] - ox) ** 2 + (Y[j0:j1, i0:i1] - oy) ** 2 <= rr ** 2
        occ[j0:j1, i0:i1] |= sub
    return edt_costmap(occ, power)


def surface_obstacles_costmap(costmap_size, half_width, obstacles, origin, r_robot, power=20):
    """Surface.create_obstacles_costmap (MPPI_isaac.py:361-378) with scipy's EDT in place of cv2.

    Frame swap x_local = y - y0, y_local = x - x0 and radius r/2 + r_robot + 0.1, as the reference.
    """
    x = np.linspace(-half_width, half_width, costmap_size)
    X, Y = np.meshgrid(x, x)
    occ = np.zeros((costmap_size, costmap_size), bool)
    x0, y0 = origin
    for xg, yg, r in obstacles:
        xl = yg - y0
        yl = xg - x0
        tr = r / 2 + r_robot + 0.1
        occ |= (X - xl) ** 2 + (Y - yl) ** 2 <= tr ** 2
    return edt_costmap(occ, power)


def scene_c3():
    """Configs C1-C4: 1500^2 DEM @0.1 m (half-width 75), 750^2 costmap @0.2 m."""
    Z = crater_dem(1500, 75.0)
    cm = disc_costmap(750, 75.0, random_obstacles())
    return Z, 75.0, cm


def _fbm_factors(grid, half_width, seed=7, octaves=5, amp=0.3, base_wavelength=8.0):
    """Seeded band-limited fBm (random sinusoid octaves) as rank-1 factors (row, column) pairs.

    sin(kx x + ky y + ph) = cos(ky y) sin(kx x + ph) + sin(ky y) cos(kx x + ph).
    """
    rng = np.random.RandomState(seed)
    x = np.linspace(-half_width, half_width, grid, dtype=np.float32)
    rows, cols = [], []
    for o in range(octaves):
        lam = base_wavelength / (2 ** o)
        a = np.float32(amp / (2 ** o))
        for _ in range(3):
            th = rng.uniform(0, np.pi)
            ph = rng.uniform(0, 2 * np.pi)
            kx = np.float32(2 * np.pi / lam * np.cos(th))
            ky = np.float32(2 * np.pi / lam * np.sin(th))
            ax = kx * x + np.float32(ph)
            by = ky * x
            rows += [a * np.cos(by), a * np.sin(by)]
            cols += [np.sin(ax), np.cos(ax)]
    return rows, cols


def _crater_factors(grid_size, half_width, bumps=BUMPS_9, scale=1.0):
    """The crater formula of MPPI_isaac.py:318-320 with each gaussian split as exp(-dy^2/2w^2) x exp(-dx^2/2w^2)."""
    x = np.linspace(-half_width, half_width, grid_size)
    rows, cols = [], []
    for (cx, cy), h, w in bumps:
        cx, cy, w = cx * scale, cy * scale, w * scale
        for amp, ww in ((h - 0.5, w), (-(h + 0.5), w / 2)):
            rows.append((amp * np.exp(-(x - cy) ** 2 / (2 * ww ** 2))).astype(np.float32))
            cols.append(np.exp(-(x - cx) ** 2 / (2 * ww ** 2)).astype(np.float32))
    return rows, cols


def fbm(grid, half_width, seed=7, octaves=5, amp=0.3, base_wavelength=8.0):
    """Seeded band-limited fBm (sum of random sinusoid octaves), for C5 roughness."""
    rows, cols = _fbm_factors(grid, half_width, seed, octaves, amp, base_wavelength)
    return np.stack(rows, 1) @ np.stack(cols, 0)


def scene_c5():
    """Config C5: 8192^2 DEM @0.025 m (half-width 102.4), craters x2 in size + fBm; 1024^2 costmap.

    The terrain is a sum of 48 separable terms (18 crater gaussians, 30 fBm sinusoids), built as
    one float32 (8192 x 48) @ (48 x 8192) product, so the tile takes a second, not ~30 s.
    """
    r1, c1 = _crater_factors(8192, 102.4, scale=4.0 / 1.0 * 0.5)
    r2, c2 = _fbm_factors(8192, 102.4)
    Z = np.stack(r1 + r2, 1) @ np.stack(c1 + c2, 0)
    cm = disc_costmap(1024, 102.4, random_obstacles(extent=90.0))
    return Z.astype(np.float32), 102.4, cm
