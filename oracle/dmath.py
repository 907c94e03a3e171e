"""Deterministic float32 math + Philox4x32-10, restated in numpy.

TEST INFRASTRUCTURE ONLY. Nothing under ``oracle/`` is imported by the product
path; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, as the checker.

Why this module exists
----------------------
The reference evaluates ``wp.sin``/``wp.cos``/``wp.exp``/``wp.randn`` with
CUDA's libdevice (projection_warp.py:236-237, critics_warp.py:347,
sampling_warp.py:73-91).  Those results cannot be reproduced offline, and the
MPPI softmax at T=0.3 (config.yaml:28) turns one-ulp cost differences into
visible control differences.  The build therefore *defines* every
transcendental as a fixed sequence of IEEE float32 +,-,*,/ operations (Cephes
minimax polynomials, no FMA contraction).  The HIP kernels
(``csrc/mppi_detmath.h``) and this numpy restatement run the same sequence, so
they agree bit for bit.

Noise: rocRAND's Philox4x32-10 (``rocrand_philox4x32_10.h``; Random123
algorithm) with key = seed and counter = (n_lo, n_hi, k_lo, k_hi), i.e. the
rocRAND state ``rocrand_init(seed, subsequence=k, offset=4*n)``.  This replaces
Warp's ``wp.randn(seed+tid+...)`` hashing (sampling_warp.py:73-91), whose
correlated streams are a documented divergence.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
U32 = np.uint32
U64 = np.uint64

# ---------------------------------------------------------------- constants
SQRTHF = F32(0.707106781186547524)
LOG_P = [F32(c) for c in (7.0376836292e-2, -1.1514610310e-1, 1.1676998740e-1,
                          -1.2420140846e-1, 1.4249322787e-1, -1.6668057665e-1,
                          2.0000714765e-1, -2.4999993993e-1, 3.3333331174e-1)]
LOG_Q1 = F32(-2.12194440e-4)
LOG_Q2 = F32(0.693359375)

LOG2EF = F32(1.44269504088896341)
EXP_C1 = F32(0.693359375)
EXP_C2 = F32(-2.12194440e-4)
EXP_P = [F32(c) for c in (1.9875691500e-4, 1.3981999507e-3, 8.3334519073e-3,
                          4.1665795894e-2, 1.6666665459e-1, 5.0000001201e-1)]
EXP_LO = F32(-87.0)

FOPI = F32(1.27323954473516)
DP1 = F32(0.78515625)
DP2 = F32(2.4187564849853515625e-4)
DP3 = F32(3.77489497744594108e-8)
SIN_P = [F32(c) for c in (-1.9515295891e-4, 8.3321608736e-3, -1.6666654611e-1)]
COS_P = [F32(c) for c in (2.443315711809948e-5, -1.388731625493765e-3,
                          4.166664568298827e-2)]
TWO_PI = F32(6.2831853071795864769)
INV_2_24 = F32(5.9604644775390625e-8)

PHILOX_M0 = U64(0xD2511F53)
PHILOX_M1 = U64(0xCD9E8D57)
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85


def f32(x):
    return np.asarray(x, dtype=F32)


# ---------------------------------------------------------------- dm_logf
def dm_logf(x):
    """Cephes logf for normal positive float32 x (csrc/mppi_detmath.h dm_logf)."""
    x = f32(x)
    bits = x.view(U32)
    e = ((bits >> U32(23)) & U32(0xFF)).astype(np.int32) - 126
    m = ((bits & U32(0x807FFFFF)) | U32(0x3F000000)).view(F32)
    small = m < SQRTHF
    e = np.where(small, e - 1, e)
    m = np.where(small, (m + m) - F32(1.0), m - F32(1.0)).astype(F32)
    z = m * m
    y = np.full_like(m, LOG_P[0])
    for c in LOG_P[1:]:
        y = y * m
        y = y + c
    y = y * m
    y = y * z
    fe = e.astype(F32)
    y = y + LOG_Q1 * fe
    y = y + F32(-0.5) * z
    r = m + y
    r = r + LOG_Q2 * fe
    return r


# ---------------------------------------------------------------- dm_expf
def dm_expf(x):
    """Cephes expf; defined as 0 for x < -87 (csrc/mppi_detmath.h dm_expf)."""
    x = f32(x)
    lo = x < EXP_LO
    xc = np.where(lo, F32(0.0), x).astype(F32)
    t = LOG2EF * xc
    t = t + F32(0.5)
    z = np.floor(t).astype(F32)
    r = xc - z * EXP_C1
    r = r - z * EXP_C2
    n = z.astype(np.int32)
    zz = r * r
    p = np.full_like(r, EXP_P[0])
    for c in EXP_P[1:]:
        p = p * r
        p = p + c
    y = p * zz
    y = y + r
    y = y + F32(1.0)
    scale = ((n + 127).astype(np.int64) << 23).astype(U32).view(F32)
    y = y * scale
    return np.where(lo, F32(0.0), y).astype(F32)


# ---------------------------------------------------------------- dm_sincosf
def dm_sincosf(x):
    """Cephes sinf/cosf with shared reduction; returns (sin, cos)."""
    x = f32(x)
    ax = np.abs(x)
    j = (ax * FOPI).astype(np.int32)
    y = j.astype(F32)
    odd = (j & 1) == 1
    j = np.where(odd, j + 1, j)
    y = np.where(odd, y + F32(1.0), y).astype(F32)
    j = j & 7
    r = ax - y * DP1
    r = r - y * DP2
    r = r - y * DP3
    z = r * r
    ps = SIN_P[0] * z
    ps = ps + SIN_P[1]
    ps = ps * z
    ps = ps + SIN_P[2]
    ps = ps * z
    ps = ps * r
    ps = ps + r
    pc = COS_P[0] * z
    pc = pc + COS_P[1]
    pc = pc * z
    pc = pc + COS_P[2]
    pc = pc * z
    pc = pc * z
    pc = pc - F32(0.5) * z
    pc = pc + F32(1.0)
    q = j >> 1
    s = np.select([q == 0, q == 1, q == 2], [ps, pc, -ps], -pc).astype(F32)
    c = np.select([q == 0, q == 1, q == 2], [pc, -ps, -pc], ps).astype(F32)
    s = np.where(x < F32(0.0), -s, s).astype(F32)
    return s, c


def dm_sincosf_small(x):
    """dm_sincosf for |x| * 4/pi < 1 without the reduction (csrc/mppi_detmath.h dm_sincosf_small):
    the same float32 op sequence on r = x; equal bits there (tests/test_oracle_golden.py)."""
    x = f32(x)
    z = x * x
    ps = SIN_P[0] * z
    ps = ps + SIN_P[1]
    ps = ps * z
    ps = ps + SIN_P[2]
    ps = ps * z
    ps = ps * x
    ps = ps + x
    pc = COS_P[0] * z
    pc = pc + COS_P[1]
    pc = pc * z
    pc = pc + COS_P[2]
    pc = pc * z
    pc = pc * z
    pc = pc - F32(0.5) * z
    pc = pc + F32(1.0)
    return ps.astype(F32), pc.astype(F32)


# ---------------------------------------------------------------- Philox
def _mulhilo(m, a):
    p = m * a.astype(U64)
    return (p >> U64(32)).astype(U32), (p & U64(0xFFFFFFFF)).astype(U32)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 block (rocrand_philox4x32_10.h ten_rounds/single_round).

    Arguments broadcast; all uint32.  Returns four uint32 arrays.
    """
    c0, c1, c2, c3 = (np.asarray(v, dtype=U32) for v in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for rnd in range(10):
        hi0, lo0 = _mulhilo(PHILOX_M0, c0)
        hi1, lo1 = _mulhilo(PHILOX_M1, c2)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ U32(k0), lo1, hi0 ^ c3 ^ U32(k1), lo0)
        k0 = (k0 + PHILOX_W0) & 0xFFFFFFFF
        k1 = (k1 + PHILOX_W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def box_muller(ra, rb):
    """Two uint32 -> two standard normals (float32), csrc dm_box_muller."""
    ra = np.asarray(ra, dtype=U32)
    rb = np.asarray(rb, dtype=U32)
    u = ((ra >> U32(8)).astype(F32) + F32(1.0)) * INV_2_24      # (0, 1]
    v = (rb >> U32(8)).astype(F32) * INV_2_24                  # [0, 1)
    rad = np.sqrt(F32(-2.0) * dm_logf(u)).astype(F32)
    s, c = dm_sincosf(TWO_PI * v)
    return rad * c, rad * s


def noise_block(seed, n, k):
    """Four normals for block n of trajectory k: (e1[t], e2[t], e1[t+1], e2[t+1]).

    Counter = (n lo, n hi, k lo, k hi), key = seed (lo, hi).
    """
    seed = int(seed)
    n = int(n)
    k = np.asarray(k, dtype=np.int64)
    r0, r1, r2, r3 = philox4x32_10(U32(n & 0xFFFFFFFF), U32((n >> 32) & 0xFFFFFFFF),
                                   (k & 0xFFFFFFFF).astype(U32), (k >> 32).astype(U32),
                                   seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    z0, z1 = box_muller(r0, r1)
    z2, z3 = box_muller(r2, r3)
    return z0, z1, z2, z3


def noise(seed, step, k, H):
    """Noise matrices eps1, eps2 of shape [len(k), H] for MPPI step ``step``.

    Block index n = step * ceil(H/2) + t//2 (t even).
    """
    k = np.atleast_1d(np.asarray(k, dtype=np.int64))
    hp = (H + 1) // 2
    e1 = np.empty((k.size, H), F32)
    e2 = np.empty((k.size, H), F32)
    for tp in range(hp):
        z0, z1, z2, z3 = noise_block(seed, int(step) * hp + tp, k)
        t = 2 * tp
        e1[:, t] = z0
        e2[:, t] = z1
        if t + 1 < H:
            e1[:, t + 1] = z2
            e2[:, t + 1] = z3
    return e1, e2
