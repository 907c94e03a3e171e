"""GPU: mppi_group, the K-sharded step driven from one process (include/mppi.h).

Members sharing one device exchange their records by device copies (the path this 1-GPU box
runs); distinct devices use RCCL's ncclAllGather (run only where >= 2 GPUs are visible).  A
power-of-two leaf split is bitwise equal to one context over all K (the combine tree is the same
tree); a ragged split with an empty member equals the oracle's world-n combine bit for bit.
"""
import numpy as np
import pytest

import helpers as hp
from oracle import mppi_ref as R

pytestmark = pytest.mark.gpu


def _group(K, H, devices, Z, hw, cm, st, seed=42):
    from mppi_amd import _lib
    g = _lib.Group(_lib.make_params(K, H, seed=seed), devices)
    g.set_dem(Z, hw)
    g.set_costmap(cm, hw)
    g.set_state(hp.state_for(st))
    return g


def _same(a, b, what):
    for k in ("u1_opt", "u2_opt", "lin_vel", "ang_vel", "traj_sim", "heading_sim", "left_wheel_sim",
              "right_wheel_sim"):
        assert np.array_equal(a[k], b[k]), f"{what}: " + hp.mismatch_report(k, a[k], b[k])


@pytest.mark.parametrize("n", [1, 2])
def test_group_on_one_device_bitwise_equals_one_context(n):
    """K = 131072 (the C4 shard size) split over n members on device 0: three chained steps give
    the single context's outputs, costs and nominal controls bit for bit."""
    K, H = 131072, 24
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state()
    one = hp.engine_for(K, H, Z, hw, cm, st)
    g = _group(K, H, [0] * n, Z, hw, cm, st)
    assert [g.shard(i) for i in range(n)] == R.shard_bounds(K, n)
    try:
        for it in range(3):
            _same(g.step("3d", it), one.step("3d", it), f"step {it}")
            assert np.array_equal(g.costs(), one.costs())
        for m in g.members:
            for a, b in zip(m.get_nominal(), one.get_nominal()):
                assert np.array_equal(a, b)
    finally:
        g.close()
        one.close()


def test_group_ragged_with_empty_member_matches_oracle():
    """K = 1280 over 4 members (member 3 owns no trajectory and contributes the empty record):
    equal to the oracle's 4-shard combine, every member ending on the same nominal controls."""
    K, H, n = 1280, 12, 4
    assert R.shard_bounds(K, n)[3] == (1280, 0)
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state()
    g = _group(K, H, [0] * n, Z, hw, cm, st)
    try:
        out = g.step("3d", 2)
        u = np.zeros(H, np.float32)
        ref = R.mppi_step(R.Params(K=K, H=H, seed=42), R.Scene(Z, hw, cm), st, u, u, 2, world=n)
        np.testing.assert_array_equal(out["u1_opt"], ref["u1_opt"])
        np.testing.assert_array_equal(out["u2_opt"], ref["u2_opt"])
        np.testing.assert_array_equal(out["lin_vel"], ref["v_opt"])
        np.testing.assert_array_equal(out["traj_sim"], ref["traj_sim"])
        np.testing.assert_array_equal(g.costs(), ref["cost"])
        noms = [m.get_nominal() for m in g.members]
        for u1, u2 in noms[1:]:
            assert np.array_equal(u1, noms[0][0]) and np.array_equal(u2, noms[0][1])
    finally:
        g.close()


def test_group_rccl_exchange_one_member(monkeypatch):
    """MPPI_GROUP_RCCL=1 routes even one member through partial step -> ncclAllGather -> finish
    (the RCCL exchange a 1-GPU host can run); bitwise equal to one context."""
    monkeypatch.setenv("MPPI_GROUP_RCCL", "1")
    K, H = 131072, 24
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state()
    one = hp.engine_for(K, H, Z, hw, cm, st)
    g = _group(K, H, [0], Z, hw, cm, st)
    try:
        for it in range(3):
            _same(g.step("3d", it), one.step("3d", it), f"step {it}")
    finally:
        g.close()
        one.close()


def test_group_rccl_across_devices():
    """Distinct devices: the records travel by ncclAllGather; bitwise equal to one context."""
    import torch
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 visible GPUs (the RCCL exchange)")
    n = min(n, 8)
    K, H = 65536 * n, 24
    Z, hw, cm = hp.c3_scene()
    st = hp.oracle_state()
    one = hp.engine_for(K, H, Z, hw, cm, st)
    g = _group(K, H, list(range(n)), Z, hw, cm, st)
    try:
        for it in range(2):
            _same(g.step("3d", it), one.step("3d", it), f"step {it}")
    finally:
        g.close()
        one.close()


def test_group_rejects_bad_arguments():
    from mppi_amd import _lib
    with pytest.raises(RuntimeError, match="group"):
        _lib.Group(_lib.make_params(1024, 8), [])
