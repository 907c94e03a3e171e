"""GPU: the standalone DEM lookups vs the oracle, bit for bit.

mppi_bilinear_query (scattered queries, corners gathered through L1/L2) and the
LDS-tiled path (mppi_bin_queries + mppi_bilinear_tiled) must both equal the
restatement of projection_warp.py:8-100 on the same points, including points
outside the map (clamped, DEFINED) and negative coordinates (trunc quirk).
"""
import numpy as np
import pytest

import helpers as hp
from oracle import mppi_ref as R

pytestmark = pytest.mark.gpu


def _oracle_heights(Z, hw, x, y):
    sc = R.Scene(Z, hw, np.zeros((4, 4), np.float32))
    q = R.get_corners_heights(sc, x, y)
    return R.bilinear(x, y, q, sc.res)


def _points(n, hw, seed, margin=1.5):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-hw * margin, hw * margin, n).astype(np.float32)
    y = rng.uniform(-hw * margin, hw * margin, n).astype(np.float32)
    x[:8] = np.array([0.0, -0.0, hw, -hw, 1e-30, -1e-30, 0.05, -0.05], np.float32)   # edges, tiny, zero
    y[:8] = np.array([0.0, 0.0, -hw, hw, -1e-30, 1e-30, -0.05, 0.05], np.float32)
    return x, y


def _engine(Z, hw):
    from mppi_amd import _lib
    eng = _lib.Engine(_lib.make_params(256, 8), 0)
    eng.set_dem(Z, hw)
    return eng


@pytest.mark.parametrize("which", ["c3", "odd", "few_tiles"])
def test_bilinear_query_and_tiled_match_oracle(which):
    import torch
    if which == "odd":   # ragged map: rows/cols not multiples of the 128-cell tile
        rng = np.random.default_rng(3)
        Z = rng.normal(size=(203, 203)).astype(np.float32)
        hw = 10.15
    else:
        Z, hw, _ = hp.c3_scene()
    n = 200_003
    x, y = _points(n, hw, seed=11)
    if which == "few_tiles":   # every query in 4 tiles: long runs per sorted block
        x = (x % np.float32(5.0)).astype(np.float32)
        y = (y % np.float32(5.0)).astype(np.float32)
    want = _oracle_heights(Z, hw, x, y)
    eng = _engine(Z, hw)
    xd = torch.from_numpy(x).cuda()
    yd = torch.from_numpy(y).cuda()
    hd = torch.empty_like(xd)
    eng.bilinear_query(xd.data_ptr(), yd.data_ptr(), hd.data_ptr(), n)
    got = hd.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32)), \
        hp.mismatch_report("bilinear_query", got, want)

    nt = eng.bilinear_tiles()
    xs = torch.empty_like(xd)
    ys = torch.empty_like(xd)
    perm = torch.empty(n, dtype=torch.int32, device="cuda")
    off = torch.empty(nt + 1, dtype=torch.int32, device="cuda")
    eng.bin_queries(xd.data_ptr(), yd.data_ptr(), n, xs.data_ptr(), ys.data_ptr(), perm.data_ptr(), off.data_ptr())
    o = off.cpu().numpy()
    assert o[0] == 0 and o[-1] == n and np.all(np.diff(o) >= 0)
    p = perm.cpu().numpy()
    assert np.array_equal(np.sort(p), np.arange(n))
    assert np.array_equal(xs.cpu().numpy(), x[p]) and np.array_equal(ys.cpu().numpy(), y[p])
    ht = torch.empty_like(xd)
    eng.bilinear_tiled(xs.data_ptr(), ys.data_ptr(), off.data_ptr(), ht.data_ptr())
    eng.sync()
    tiled = np.empty(n, np.float32)
    tiled[p] = ht.cpu().numpy()
    assert np.array_equal(tiled.view(np.uint32), got.view(np.uint32)), hp.mismatch_report("tiled", tiled, got)
    eng.close()


def test_bin_queries_empty():
    import torch
    Z = np.zeros((64, 64), np.float32)
    eng = _engine(Z, 3.2)
    nt = eng.bilinear_tiles()
    assert nt == 1
    e = torch.empty(1, device="cuda")   # valid pointers; n = 0
    off = torch.full((nt + 1,), -1, dtype=torch.int32, device="cuda")
    perm = torch.empty(1, dtype=torch.int32, device="cuda")
    eng.bin_queries(e.data_ptr(), e.data_ptr(), 0, e.data_ptr(), e.data_ptr(), perm.data_ptr(), off.data_ptr())
    assert off.cpu().tolist() == [0, 0]
    eng.close()


def test_bin_queries_refuses_skinny_dem():
    """A skinny DEM (2 x 2^23 cells: 65 536 tiles of 128 x 128) has more tiles than the binning's LDS
    histogram holds: mppi_bin_queries refuses it with a clear error instead of a failed launch."""
    import torch
    Z = np.zeros((2, 1 << 23), np.float32)
    eng = _engine(Z, 3.2)
    assert eng.bilinear_tiles() == 65536
    e = torch.empty(4, device="cuda")
    perm = torch.empty(4, dtype=torch.int32, device="cuda")
    off = torch.empty(65537, dtype=torch.int32, device="cuda")
    with pytest.raises(RuntimeError, match="exceed the LDS histogram"):
        eng.bin_queries(e.data_ptr(), e.data_ptr(), 4, e.data_ptr(), e.data_ptr(), perm.data_ptr(), off.data_ptr())
    eng.close()
