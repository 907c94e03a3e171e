"""TEST INFRASTRUCTURE ONLY — the reference's numpy 2.5D integrator, batched over K trajectories.

Restates thesis_master/python_mppi_projection/debug.py:170-364 (generate_trajectory_25D and its
helpers) in float64, vectorised over trajectories; the checker for the HIP "python25d" integrator
(csrc/mppi_python25d.hip).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.

Differences from the Warp rollout (projection_warp.py:284-350) that this mode keeps on purpose:
  * the heading is rotated about the PREVIOUS normal before the new cell is looked up
    (debug.py:352-357), and the step's displacement uses the normalised heading (:278-282);
  * cell indices come from np.searchsorted on the linspace grid X[0] / Y[:, 0] (:186-190), whose
    spacing 2hw/(grid-1) differs from `resolution` = 2hw/grid; rows grow with y (Y ascending);
  * bilinear fractions use floor, not trunc (:246-250);
  * a trajectory that leaves |x|, |y| < bound (20 m in debug.py:359) is discarded (returns None).
"""
from __future__ import annotations

import numpy as np


def linspace_grid(half_width, n):
    """np.linspace(-hw, hw, n) (the X[0] / Y[:, 0] axis of debug.py's meshgrid)."""
    return np.linspace(-half_width, half_width, n)


def corners(x, y, res, xs, ys, Z):
    """find_corners_heights (debug.py:170-198): q[:, a, b] for K points.

    DEFINED: i, j are clamped to [0, grid-2]; the reference raises IndexError (or wraps a negative
    index) there, e.g. for x in [19.9, 20) on its 400^2 / 20 m scene.
    """
    x0 = np.floor(x / res) * res
    y0 = np.floor(y / res) * res
    i = np.clip(np.searchsorted(xs, x0), 0, Z.shape[1] - 2)
    j = np.clip(np.searchsorted(ys, y0), 0, Z.shape[0] - 2)
    q = np.empty((x.shape[0], 2, 2))
    q[:, 0, 0] = Z[j, i]
    q[:, 0, 1] = Z[j, i + 1]
    q[:, 1, 0] = Z[j + 1, i]
    q[:, 1, 1] = Z[j + 1, i + 1]
    return q


def bilinear(x, y, q, res):
    """bilinear_interpolator (debug.py:234-257)."""
    xn = x / res
    yn = y / res
    x2 = xn - np.floor(xn)
    y2 = yn - np.floor(yn)
    return ((1.0 - x2) * (1.0 - y2) * q[:, 0, 0] + x2 * (1.0 - y2) * q[:, 1, 0]
            + (1.0 - x2) * y2 * q[:, 0, 1] + x2 * y2 * q[:, 1, 1])


def _norm(v):
    return np.sqrt(v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2])[:, None]


def normal_on_grid(q, g):
    """debug.py:200-216."""
    v = np.stack([-g / 2.0 * (q[:, 0, 1] - q[:, 0, 0] - q[:, 1, 0] + q[:, 1, 1]),
                  -g / 2.0 * (q[:, 1, 0] - q[:, 0, 0] - q[:, 0, 1] + q[:, 1, 1]),
                  np.full(q.shape[0], g * g)], 1)
    return v / _norm(v)


def tangent(n, h):
    """get_heading_tangent_vector (debug.py:218-232)."""
    d = (h[:, 0] * n[:, 0] + h[:, 1] * n[:, 1] + h[:, 2] * n[:, 2])[:, None]
    p = h - d * n
    return p / _norm(p)


def rotvec_apply(rv, v):
    """scipy Rotation.from_rotvec(rv).apply(v): quaternion (Taylor scale below 1e-3 rad), as_matrix, M v."""
    ang = _norm(rv)[:, 0]
    a2 = ang * ang
    small = ang <= 1e-3
    with np.errstate(invalid="ignore", divide="ignore"):
        scale = np.where(small, 0.5 - a2 / 48 + a2 * a2 / 3840, np.sin(ang / 2) / ang)
    x, y, z = (scale * rv[:, 0], scale * rv[:, 1], scale * rv[:, 2])
    w = np.cos(ang / 2)
    x2, y2, z2, w2 = x * x, y * y, z * z, w * w
    xy, zw, xz, yw, yz, xw = x * y, z * w, x * z, y * w, y * z, x * w
    m = np.empty((rv.shape[0], 3, 3))
    m[:, 0, 0] = x2 - y2 - z2 + w2
    m[:, 1, 0] = 2 * (xy + zw)
    m[:, 2, 0] = 2 * (xz - yw)
    m[:, 0, 1] = 2 * (xy - zw)
    m[:, 1, 1] = -x2 + y2 - z2 + w2
    m[:, 2, 1] = 2 * (yz + xw)
    m[:, 0, 2] = 2 * (xz + yw)
    m[:, 1, 2] = 2 * (yz - xw)
    m[:, 2, 2] = -x2 - y2 + z2 + w2
    return m[:, :, 0] * v[:, 0:1] + m[:, :, 1] * v[:, 1:2] + m[:, :, 2] * v[:, 2:3]


def generate_trajectories_25d(x0, y0, heading, v, w, dt, Z, half_width, resolution, bound=20.0):
    """generate_trajectory_25D (debug.py:312-364) for K trajectories.

    x0, y0 [K]; heading [K, 3]; v, w [K, H]; Z [grid, grid] (rows = ascending y).
    Returns traj [K, H, 3] (x, y, height) and valid [K] (False where the reference returns None;
    those rows hold the steps computed before leaving the bound, then zeros).
    """
    x = np.asarray(x0, np.float64).copy()
    y = np.asarray(y0, np.float64).copy()
    h = np.asarray(heading, np.float64).reshape(-1, 3).copy()
    v = np.asarray(v, np.float64)
    w = np.asarray(w, np.float64)
    K, H = v.shape
    Z = np.asarray(Z, np.float64)
    xs = linspace_grid(half_width, Z.shape[1])
    ys = linspace_grid(half_width, Z.shape[0])
    q = corners(x, y, resolution, xs, ys, Z)
    n = normal_on_grid(q, resolution)
    h = tangent(n, h)
    traj = np.zeros((K, H, 3))
    valid = np.ones(K, bool)
    for k in range(H):
        act = np.nonzero(valid)[0]
        if act.size == 0:
            break
        hh = h[act] / _norm(h[act])                         # update_position :278-290
        xa = x[act] + hh[:, 0] * v[act, k] * dt
        ya = y[act] + hh[:, 1] * v[act, k] * dt
        ang = w[act, k] * dt
        hr = rotvec_apply(ang[:, None] * n[act], hh)
        hr = hr / _norm(hr)
        out = (xa >= bound) | (xa <= -bound) | (ya >= bound) | (ya <= -bound)   # :359-360
        qa = corners(xa, ya, resolution, xs, ys, Z)         # :354-357
        hgt = bilinear(xa, ya, qa, resolution)
        na = normal_on_grid(qa, resolution)
        ha = tangent(na, hr)
        x[act], y[act], n[act], h[act] = xa, ya, na, ha
        keep = act[~out]
        traj[keep, k, 0] = xa[~out]
        traj[keep, k, 1] = ya[~out]
        traj[keep, k, 2] = hgt[~out]
        valid[act[out]] = False
    return traj, valid
