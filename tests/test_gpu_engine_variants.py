"""GPU: the engine's scheduling variants are bitwise identical to the default path.

Each toggle below changes only WHERE or WHEN work runs, never the arithmetic:
  MPPI_COLFIN=0     finish by the record tree (mppi_finish_kernel) instead of the
                    column-split kernel
  MPPI_UCACHE=0     leaf reduction re-reads every normals row instead of the LDS-cached controls
  MPPI_NOISE_AT=1/2 noise of the steps ahead launched after the finish / beside the rollout
  MPPI_NOISE_AHEAD=1  normals generated one step ahead instead of two
  MPPI_ROLES=0/1    the pair rollout kernel / the role-split one at any K
  MPPI_NOISE_GPC=1  noise grid of one workgroup per CU
  MPPI_FUSED=0      rollout, finish and noise as three launches instead of the fused step launch
  MPPI_FUSED=2      the fused launch also with the deferred tail (default: synchronous steps only)
  MPPI_FUSED_NOISE_GROUPS=0/7/-2  the fused launch's noise before it on the context stream / inside it
                    on 7 workgroups / after it on the noise stream behind a gate kernel (default:
                    inside it on one workgroup per CU the finish leaves)
  MPPI_WAVE_PRIO=0  rollout waves at the default issue priority (no s_setprio)
The toggles are read when a context is created, so each variant gets its own engine.
Sizes: n = 256 leaf records (C3 K) and n = 1024 (C5 K) at a short horizon.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ("u1_opt", "u2_opt", "lin_vel", "ang_vel")


def _run(env, K, H, steps=3, info=None, step_ids=None):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mppi_amd import _lib, scene
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        eng = _lib.Engine(_lib.make_params(K, H), 0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    Z, hw, cm = scene.scene_c3()
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
    outs = []
    for i in (step_ids if step_ids is not None else range(steps)):
        o = eng.step("3d", i)
        outs.append({k: o[k].copy() for k in KEYS})
    costs = eng.costs()
    if info is not None:
        info.update(eng.launch_info())
    eng.close()
    return outs, costs


@pytest.mark.parametrize("K,H", [(65536, 24), (262144, 16)])
@pytest.mark.parametrize("env", [{"MPPI_COLFIN": "0"}, {"MPPI_UCACHE": "0"}, {"MPPI_NOISE_AT": "1"},
                                 {"MPPI_NOISE_AT": "2"}, {"MPPI_NOISE_AHEAD": "1"}, {"MPPI_ROLES": "0"},
                                 {"MPPI_ROLES": "1"}, {"MPPI_NOISE_GPC": "1"}, {"MPPI_FUSED": "0"},
                                 {"MPPI_FUSED": "2"}, {"MPPI_FUSED_NOISE_GROUPS": "0"},
                                 {"MPPI_FUSED_NOISE_GROUPS": "7"}, {"MPPI_FUSED_NOISE_GROUPS": "-2"},
                                 {"MPPI_WAVE_PRIO": "0"}],
                         ids=["record-tree", "no-ucache", "noise-after-finish", "noise-beside-rollout",
                              "noise-one-ahead", "pair-kernel", "role-split-kernel", "noise-1-per-cu",
                              "unfused", "fused-pipelined-too", "fused-noise-separate", "fused-7-noise-groups",
                              "fused-noise-gated", "no-wave-priority"])
def test_variant_bitwise_equal(K, H, env):
    ref, ref_costs = _run({}, K, H)
    got, got_costs = _run(env, K, H)
    np.testing.assert_array_equal(got_costs, ref_costs)
    for i, (a, b) in enumerate(zip(got, ref)):
        for k in KEYS:
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"step {i} {k} {env}")


@pytest.mark.parametrize("K,H", [(1048576, 40), (1048576, 100)])
def test_column_split_finish_at_4096_records(K, H):
    """n = 4096 leaf records: the column-split finish's levels above one wave (H=40), and the
    record-tree fallback where (columns + 1) x (records / 16) exceeds the workgroup (H=100).
    launch_info names the finish that ran; the oracle pins H=100 in test_gpu_headline.py."""
    i_ref, i_got = {}, {}
    ref, ref_costs = _run({"MPPI_COLFIN": "0"}, K, H, steps=2, info=i_ref)
    got, got_costs = _run({}, K, H, steps=2, info=i_got)
    assert i_ref["finish_kind"] == 0 and i_ref["finish_records"] == 4096
    assert i_got["finish_kind"] == (1 if H == 40 else 0), i_got
    if H == 40:
        assert i_got["finish_records"] == 4096 and i_got["finish_ncol"] >= 2
    np.testing.assert_array_equal(got_costs, ref_costs)
    for i, (a, b) in enumerate(zip(got, ref)):
        for k in KEYS:
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"step {i} {k}")


@pytest.mark.parametrize("env", [{"MPPI_FUSED": "0"}, {"MPPI_FUSED": "1"}], ids=["unfused", "fused"])
def test_step_counter_jumps(env):
    """Step counters that skip and repeat (normals generated out of order, slots reused) give the
    same results with and without the fused launch."""
    ids = [0, 1, 5, 6, 6, 2]
    ref, ref_costs = _run({"MPPI_FUSED": "0", "MPPI_ROLES": "0"}, 65536, 24, step_ids=ids)
    got, got_costs = _run(env, 65536, 24, step_ids=ids)
    np.testing.assert_array_equal(got_costs, ref_costs)
    for i, (a, b) in enumerate(zip(got, ref)):
        for k in KEYS:
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"call {i} {k} {env}")


def test_timing_modes():
    """mppi_set_timing: mode 2 times the rollout only (no host wait), mode 1 also the finish and
    the deferred tail; other modes are refused."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mppi_amd import _lib, scene
    eng = _lib.Engine(_lib.make_params(65536, 24), 0)
    Z, hw, cm = scene.scene_c3()
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
    try:
        eng.set_async_tail(True)
        eng.set_timing(2)
        for i in range(4):
            eng.step("3d", i, copy=False)
        roll, fin, n = eng.timing()
        assert n == 4 and roll > 0.0 and fin == 0.0
        assert eng.tail_timing()[1] == 0
        eng.set_timing(True)
        for i in range(4, 8):
            eng.step("3d", i, copy=False)
        roll, fin, n = eng.timing()
        fused = eng.launch_info()["fused"] == 1   # a fused launch times rollout + finish as one kernel
        assert n == 4 and roll > 0.0 and (fin == 0.0 if fused else fin > 0.0)
        assert eng.tail_timing()[1] >= 3
        with pytest.raises(Exception):
            eng.set_timing(3)
    finally:
        eng.close()


def test_fused_finish_gives_up_then_recovers():
    """A fused finish that stops waiting for the records (mppi_set_option("fused_wait_ticks", 0):
    give up at once) publishes nothing: the step raises, the host re-arms the record and handoff
    counters, and the next step is bitwise equal to a fresh context's (the nominal controls were
    not touched by the failed step)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mppi_amd import _lib, scene
    Z, hw, cm = scene.scene_c3()

    def make():
        e = _lib.Engine(_lib.make_params(65536, 24), 0)
        e.set_dem(Z, hw)
        e.set_costmap(cm, hw)
        e.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
        return e

    eng, ref = make(), make()
    try:
        eng.set_option("fused_wait_ticks", 0)
        with pytest.raises(RuntimeError, match="without publishing"):
            eng.step("3d", 0)
        assert eng.launch_info()["fused"] == 1
        eng.set_option("fused_wait_ticks", 200000000)
        for i in (1, 2):
            a, b = eng.step("3d", i), ref.step("3d", i)
            for k in KEYS:
                np.testing.assert_array_equal(a[k], b[k], err_msg=f"step {i} {k}")
        np.testing.assert_array_equal(eng.costs(), ref.costs())
        with pytest.raises(RuntimeError, match="unknown option"):
            eng.set_option("no_such_option", 1)
    finally:
        eng.close()
        ref.close()
