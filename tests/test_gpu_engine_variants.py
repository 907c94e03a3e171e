"""GPU: the engine's schedules are bitwise identical to each other.

Each variant below changes only WHERE or WHEN work runs, never the arithmetic:
  resident server (default)  sampled steps of the role-split plan on one resident launch
                             (mppi_step_server_kernel)
  "resident" = 0             one launch per kernel: rollout, column-split finish, deferred tail
  MPPI_ROLES=0 / 1           the pair rollout kernel / the role-split one at any K
  "record_tree_finish" = 1   the record-tree finish (mppi_finish_kernel) instead of the column split
and the server's own protocol: idle exit and relaunch, stop by another call, a finish that gives
up, two contexts taking turns on one device, step counters that jump.
Sizes: n = 256 leaf records (C3 K) and n = 1024 (C5 K) at a short horizon.
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ("u1_opt", "u2_opt", "lin_vel", "ang_vel")
ALL = KEYS + ("traj_sim", "heading_sim", "left_wheel_sim", "right_wheel_sim")


def _engine(K, H, env=None, opts=None, async_tail=False):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mppi_amd import _lib, scene
    env = env or {}
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
    # (the server tests run it on every step, "resident" 2: with the default 1 a host gap between
    # steps longer than half the idle limit runs a step as separate launches, test_cadence_policy)
    for k, v in dict({"resident": 2}, **(opts or {})).items():
        eng.set_option(k, v)
    Z, hw, cm = scene.scene_c3()
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(-60.0, -5.0, (1.0, 0.0, 0.0), goal_x=65.0, goal_y=10.0))
    eng.set_async_tail(async_tail)
    return eng


def _state(i):
    """A different robot state per step (the closed loop's: pose, heading, wheel speeds, sigmas)."""
    from mppi_amd import _lib
    return _lib.make_state(-60.0 + 0.7 * i, -5.0 + 0.3 * i, (1.0, 0.1 * i, 0.0), left_wheel_speed=0.1 * i,
                           right_wheel_speed=0.15 * i, goal_x=65.0, goal_y=10.0, std_dev_u1=0.25 + 0.05 * i,
                           std_dev_u2=0.4)


def _run(K, H, env=None, opts=None, steps=3, info=None, step_ids=None, async_tail=False, states=False):
    eng = _engine(K, H, env, opts, async_tail)
    outs = []
    try:
        for n, i in enumerate(step_ids if step_ids is not None else range(steps)):
            if states:
                eng.set_state(_state(n))
            eng.step("3d", i, copy=False)
            o = eng.outputs()
            outs.append({k: o[k].copy() for k in ALL})
        costs = eng.costs()
        if info is not None:
            info.update(eng.launch_info())
    finally:
        eng.close()
    return outs, costs


def _same(got, ref, tag):
    (g, gc), (r, rc) = got, ref
    np.testing.assert_array_equal(gc, rc, err_msg=f"costs {tag}")
    for i, (a, b) in enumerate(zip(g, r)):
        for k in ALL:
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"step {i} {k} {tag}")


@pytest.mark.parametrize("K,H", [(65536, 24), (262144, 16)])
@pytest.mark.parametrize("variant", ["separate-launches", "noise-after-rollout", "noise-after-finish", "pair-kernel",
                                     "role-split-kernel", "record-tree"])
def test_variant_bitwise_equal(K, H, variant):
    env, opts = {}, {}
    if variant == "separate-launches":
        opts = {"resident": 0}
    elif variant.startswith("noise-after"):  # the next steps' noise ordered after the rollout / the finish
        opts = {"resident": 0, "eps_after": 0 if variant.endswith("rollout") else 1}
    elif variant == "pair-kernel":
        env = {"MPPI_ROLES": "0"}
    elif variant == "role-split-kernel":
        env = {"MPPI_ROLES": "1"}
    else:
        opts = {"record_tree_finish": 1}
    i_ref, i_got = {}, {}
    ref = _run(K, H, info=i_ref)
    got = _run(K, H, env, opts, info=i_got)
    _same(got, ref, variant)
    if K == 65536:  # the default at C3 is the server; at 1024 records the pair kernel, separate launches
        assert i_ref["resident"] == 1 and i_ref["server_steps"] == 3, i_ref
    else:
        assert i_ref["resident"] == 0, i_ref
    if variant != "role-split-kernel":
        assert i_got["resident"] == 0, i_got


@pytest.mark.parametrize("async_tail", [False, True], ids=["sync", "deferred-tail"])
def test_server_closed_loop_states(async_tail):
    """A new robot state every step (the command block carries it), with and without the deferred
    optimal rollout: the server equals the separate launches in every output, incl. the *_sim rows."""
    i_got = {}
    ref = _run(65536, 24, opts={"resident": 0}, steps=5, async_tail=async_tail, states=True)
    # (an idle limit far above this loop's host work between steps: one launch serves all five)
    got = _run(65536, 24, opts={"resident_idle_us": 5000}, steps=5, async_tail=async_tail, states=True, info=i_got)
    _same(got, ref, f"closed loop async={async_tail}")
    assert i_got["resident"] == 1 and i_got["server_launches"] == 1 and i_got["server_steps"] == 5, i_got


@pytest.mark.parametrize("K", [2048, 8192, 16384])
@pytest.mark.parametrize("async_tail", [False, True], ids=["sync", "deferred-tail"])
def test_server_few_records(K, async_tail):
    """Few leaf records (8 / 32 / 64): every rollout workgroup may hold a finish column, so the
    normals of step + 2 come from the noise kernel instead of the server's noise phase (8 and 32
    records) or from the few workgroups outside the finish (64).  Five steps with the nominal
    sequence carried across them equal the separate launches."""
    i_got = {}
    ref = _run(K, 40, opts={"resident": 0}, steps=5, async_tail=async_tail, states=True)
    got = _run(K, 40, steps=5, async_tail=async_tail, states=True, info=i_got)
    _same(got, ref, f"K={K} async={async_tail}")
    assert i_got["resident"] == 1 and i_got["server_steps"] == 5, i_got


def test_server_idle_exit_and_stop():
    """The server leaves after its idle limit and is relaunched by the next step; a call that stops it
    (mppi_get_costs) between steps, too.  Every step equals the separate launches."""
    ref = _run(65536, 24, opts={"resident": 0}, steps=4, async_tail=True)
    eng = _engine(65536, 24, opts={"resident_idle_us": 5000}, async_tail=True)
    outs = []
    try:
        for i in range(4):
            eng.step("3d", i, copy=False)
            o = eng.outputs()
            outs.append({k: o[k].copy() for k in ALL})
            if i == 1:
                time.sleep(0.02)      # past the idle limit: the server has exited
            if i == 2:
                eng.costs()           # stops the server
        info = eng.launch_info()
        costs = eng.costs()
    finally:
        eng.close()
    _same((outs, costs), ref, "idle / stop")
    assert info["server_launches"] == 3 and info["server_steps"] == 4, info


def test_two_contexts_take_turns():
    """Two contexts on one device stepping alternately, each with its own server: a server waits for
    the CUs the other's holds until that one's idle exit (at most resident_idle_us).  Both equal
    their separate-launch runs."""
    ref_a = _run(65536, 24, opts={"resident": 0}, steps=3)
    ref_b = _run(32768, 20, opts={"resident": 0}, steps=3)
    a = _engine(65536, 24, opts={"resident_idle_us": 500})
    b = _engine(32768, 20, opts={"resident_idle_us": 500})
    oa, ob = [], []
    try:
        for i in range(3):
            for eng, outs in ((a, oa), (b, ob)):
                eng.step("3d", i, copy=False)
                o = eng.outputs()
                outs.append({k: o[k].copy() for k in ALL})
        ca, cb = a.costs(), b.costs()
    finally:
        a.close()
        b.close()
    _same((oa, ca), ref_a, "context a")
    _same((ob, cb), ref_b, "context b")


@pytest.mark.parametrize("K,H", [(1048576, 40), (1048576, 100)])
def test_column_split_finish_at_4096_records(K, H):
    """n = 4096 leaf records: the column-split finish's levels above one wave (H=40), and the
    record-tree fallback where (columns + 1) x (records / 16) exceeds the workgroup (H=100).
    launch_info names the finish that ran; the oracle pins H=100 in test_gpu_headline.py."""
    i_ref, i_got = {}, {}
    ref = _run(K, H, opts={"record_tree_finish": 1}, steps=2, info=i_ref)
    got = _run(K, H, steps=2, info=i_got)
    assert i_ref["finish_kind"] == 0 and i_ref["finish_records"] == 4096
    assert i_got["finish_kind"] == (1 if H == 40 else 0), i_got
    if H == 40:
        assert i_got["finish_records"] == 4096 and i_got["finish_ncol"] >= 2
    _same(got, ref, "4096 records")


@pytest.mark.parametrize("resident", [0, 1, 2], ids=["separate", "cadence", "server"])
def test_step_counter_jumps(resident):
    """Step counters that skip and repeat (normals generated out of order, slots reused) give the
    same results on the server and on separate launches of either rollout kernel."""
    ids = [0, 1, 5, 6, 6, 2]
    ref = _run(65536, 24, env={"MPPI_ROLES": "0"}, step_ids=ids, async_tail=True)
    got = _run(65536, 24, opts={"resident": resident}, step_ids=ids, async_tail=True)
    _same(got, ref, f"jumps resident={resident}")


def test_option_validation():
    """mppi_set_option refuses values outside each option's range (the context keeps its setting)."""
    eng = _engine(2048, 8)
    try:
        for name, bad in (("resident", 3), ("resident", -1), ("eps_after", 2), ("eps_after", -2),
                          ("resident_idle_us", 50), ("finish_wait_ticks", -1), ("no_such_option", 1)):
            with pytest.raises(RuntimeError, match="mppi_set_option"):
                eng.set_option(name, bad)
        for name, good in (("resident", 0), ("eps_after", -1), ("eps_after", 0), ("eps_after", 1)):
            eng.set_option(name, good)
        eng.step("3d", 0, copy=False)
    finally:
        eng.close()


def test_timing_modes():
    """mppi_set_timing: mode 2 times the rollout only (no host wait), mode 1 also the finish and
    the deferred tail (both as separate launches: timing is off the server); other modes are
    refused."""
    eng = _engine(65536, 24, async_tail=True)
    try:
        eng.set_timing(2)
        for i in range(4):
            eng.step("3d", i, copy=False)
        roll, fin, n = eng.timing()
        assert n == 4 and roll > 0.0 and fin == 0.0
        assert eng.tail_timing()[1] == 0
        assert eng.launch_info()["resident"] == 0
        eng.set_timing(True)
        for i in range(4, 8):
            eng.step("3d", i, copy=False)
        roll, fin, n = eng.timing()
        assert n == 4 and roll > 0.0 and fin > 0.0
        assert eng.tail_timing()[1] >= 3
        with pytest.raises(Exception):
            eng.set_timing(3)
    finally:
        eng.close()


def test_server_finish_gives_up_then_falls_back():
    """A server finish that stops waiting for the records (mppi_set_option("finish_wait_ticks", 0):
    give up at once) publishes the failure: the host stops the server, waits for it to retire,
    re-arms the record and handoff counters and runs the step again as separate launches, so the
    call returns the same outputs as a fresh context (counted in launch_info["server_fallbacks"]);
    with the bound restored the next steps run on the server again, still bitwise equal."""
    eng, ref = _engine(65536, 24, async_tail=True), _engine(65536, 24, opts={"resident": 0}, async_tail=True)
    try:
        eng.set_option("finish_wait_ticks", 0)
        for i in range(4):
            if i == 2:
                eng.set_option("finish_wait_ticks", 200000000)
            eng.step("3d", i, copy=False)
            ref.step("3d", i, copy=False)
            a, b = eng.outputs(), ref.outputs()
            for k in ALL:
                np.testing.assert_array_equal(a[k], b[k], err_msg=f"step {i} {k}")
            info = eng.launch_info()
            assert info["resident"] == (1 if i >= 2 else 0), (i, info)
        assert info["server_failed_steps"] == 2 and info["server_fallbacks"] == 2, info
        assert info["server_steps"] == 4, info
        np.testing.assert_array_equal(eng.costs(), ref.costs())
        with pytest.raises(RuntimeError, match="unknown option"):
            eng.set_option("no_such_option", 1)
        with pytest.raises(RuntimeError, match="resident must be"):
            eng.set_option("resident", 3)
    finally:
        eng.close()
        ref.close()


def test_cadence_policy():
    """"resident" 1 (the default): back-to-back calls run on the server, a call more than half the idle
    limit after the last step returned (a simulator frame) runs as separate launches and lets the server
    go (launch_info["cadence_steps"]); after such a step the server starts again with the second
    back-to-back call in a row, or at once when the last step ran on a server that another call
    stopped (sync).  Every step equals the separate launches."""
    ref = _run(65536, 24, opts={"resident": 0}, steps=10, async_tail=True, states=True)
    # (an idle limit of 1 ms: half of it leaves room for this loop's host work between calls)
    eng = _engine(65536, 24, opts={"resident": 1, "resident_idle_us": 1000}, async_tail=True)
    outs, sched = [], []
    try:
        for i in range(10):
            if i in (3, 6):
                time.sleep(0.005)  # a frame gap (10x half the idle limit)
            if i == 9:
                eng.sync()  # stops the server that ran step 8
            eng.set_state(_state(i))
            eng.step("3d", i, copy=False)
            sched.append(eng.launch_info()["resident"])
            o = eng.outputs()
            outs.append({k: o[k].copy() for k in ALL})
        info = eng.launch_info()
        costs = eng.costs()
    finally:
        eng.close()
    _same((outs, costs), ref, "cadence policy")
    # step 0 has no previous return; 3 and 6 follow a frame gap; 1, 4, 7 are the first back-to-back
    # call after a separate-launch step, 2, 5, 8 the second; 9 restarts the server a sync stopped
    assert sched == [0, 0, 1, 0, 0, 1, 0, 0, 1, 1], sched
    assert info["cadence_steps"] == 10 - sum(sched) and info["server_failed_steps"] == 0, info


def _hold(groups, lds, us):
    """Another stream's kernels holding CUs: `groups` workgroups with `lds` bytes of LDS each for `us`."""
    import torch
    from mppi_amd import _lib
    s = torch.cuda.Stream()
    _lib.debug_hold(0, s.cuda_stream, groups, lds, us)
    return s


def test_step_posted_under_cu_contention():
    """a step posted while another stream's kernels hold CUs.  (a) Every CU holds a
    96 KiB workgroup for 10 ms when the server is launched: none of its workgroups fits until they
    leave (nothing of the server runs, so nothing waits), and the step completes late on the server,
    bitwise equal.  (b) 16 CUs are held for 10 ms and the finish waits at most 0.5 ms for the records:
    16 of the server's workgroups cannot start (the others hold their CUs, polling for the next step),
    its finish gives up, the host stops the server (the late workgroups then run on the CUs the others
    left and it retires) and reruns the step as separate launches: no exception, bitwise equal, counted
    in launch_info["server_fallbacks"], in about the wait bound instead of the 10 ms hold."""
    import torch
    ref = _run(65536, 100, opts={"resident": 0}, steps=4, async_tail=True, states=True)
    eng = _engine(65536, 100, opts={"finish_wait_ticks": 50000}, async_tail=True)   # 0.5 ms
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    outs, lat = [], []
    try:
        for i in range(4):
            eng.set_state(_state(i))
            if i in (1, 3):
                eng.sync()  # the server leaves: the next step launches one beside the holders
                _hold(cus if i == 1 else 16, 96 * 1024, 10000)
                time.sleep(0.001)  # the holders are resident before the server's launch
            t0 = time.perf_counter()
            eng.step("3d", i, copy=False)
            lat.append(time.perf_counter() - t0)
            o = eng.outputs()
            outs.append({k: o[k].copy() for k in ALL})
            if i == 1:
                info1 = eng.launch_info()
        info = eng.launch_info()
        costs = eng.costs()
        torch.cuda.synchronize()
    finally:
        eng.close()
    _same((outs, costs), ref, "contention")
    print(f"step latency ms: {[round(x * 1e3, 3) for x in lat]}; {info}")
    assert info1["resident"] == 1 and info1["server_fallbacks"] == 0, info1   # (a) late, on the server
    assert info["server_fallbacks"] == 1 and info["server_failed_steps"] == 1, info   # (b)
    assert lat[1] > 0.004, lat                      # (a) waited for the held CUs
    assert 0.0005 < lat[3] < 0.005, lat             # (b) the wait bound, the server's exit, the rerun


@pytest.mark.parametrize("trace", [False, True], ids=["plain", "host-trace"])
def test_server_leaving_as_step_is_posted_relaunches(trace):
    """A server whose head leaves just as a step is posted (the test hook
    mppi_set_option("server_exit_after", 1): the head leaves at its poll after one step, whether or
    not the next step was posted) never takes that step: only the head leaves on its own and the
    others follow its relayed stop, so nothing of the step ran.  The host sees the launch retire
    without a completion word and relaunches the server with the same command: the step completes,
    counted in launch_info["server_relaunches"], the server stays the schedule, and every output
    equals the separate launches.  The same with MPPI_HOST_TRACE (the diagnostic path).  The idle
    limit is raised so that the host's own liveness check (a server idle for half its limit is
    stopped before posting) cannot pre-empt the relaunch on a slow host step."""
    ref = _run(65536, 24, opts={"resident": 0}, steps=4, async_tail=True, states=True)
    env = {"MPPI_HOST_TRACE": "1"} if trace else {}
    eng = _engine(65536, 24, env=env, opts={"server_exit_after": 1, "resident_idle_us": 100000}, async_tail=True)
    outs = []
    try:
        for i in range(4):
            eng.set_state(_state(i))
            eng.step("3d", i, copy=False)
            o = eng.outputs()
            outs.append({k: o[k].copy() for k in ALL})
        info = eng.launch_info()
        costs = eng.costs()
    finally:
        eng.close()
    _same((outs, costs), ref, f"relaunch trace={trace}")
    assert info["resident"] == 1 and info["server_relaunches"] == 1, info
    assert info["server_launches"] == 2 and info["server_steps"] == 4 and info["server_failed_steps"] == 0, info


def test_deferred_tail_then_partial_finish():
    """A server step leaves its optimal rollout deferred on the host (launched at the next call).  A
    partial step + finish on the same context right after it must first launch that tail, so the
    finish does not take the tail's slot while it is still to run (round-4 advisor finding).  Every
    output, the *_sim rows included, equals a context running the same calls as separate launches."""
    import torch

    def calls(opts):
        eng = _engine(65536, 24, opts=opts, async_tail=True)
        rec = torch.zeros(eng.record_len(), dtype=torch.float64, device="cuda")
        outs = []
        try:
            for i in range(4):
                eng.set_state(_state(i))
                if i in (1, 3):  # straight after a server step (no get_outputs between)
                    eng.step_partial(rec.data_ptr(), "3d", i)
                    eng.step_finish(rec.data_ptr(), 1, copy=False)
                    o = eng.outputs()
                    outs.append({k: o[k].copy() for k in ALL})
                else:
                    eng.step("3d", i, copy=False)
            costs = eng.costs()
            info = eng.launch_info()
        finally:
            eng.close()
        return (outs, costs), info

    ref, _ = calls({"resident": 0})
    got, info = calls({})
    assert info["server_steps"] == 2, info
    _same(got, ref, "deferred tail then partial + finish")
