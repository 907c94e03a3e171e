"""GPU: the armed next step (mppi_set_option "arm", include/mppi.h).

A sampled mppi_step also enqueues the next step's launches behind a gate kernel that waits for the
next call's robot state; the results must be bitwise those of the ordinary path (arm = 0) in every
way the next call can differ from the armed guess: a new state every step (the closed loop), a
step number that jumps, another call in between (cancels), a pause longer than the gate waits
(expires).  Oracle parity of the step itself is covered by test_gpu_parity / test_gpu_golden; this
file pins arm = 1 against arm = 0 on the same inputs.
"""
import time

import numpy as np
import pytest

import helpers as hp

pytestmark = pytest.mark.gpu

K, H = 8192, 40
KEYS = ("u1_opt", "u2_opt", "lin_vel", "ang_vel", "traj_sim", "heading_sim", "left_wheel_sim", "right_wheel_sim")


def _states(n):
    """A moving robot: the state the caller sets before each step."""
    out = []
    for i in range(n):
        th = 0.05 * i
        out.append(hp.oracle_state(x=-60.0 + 0.3 * i, y=-5.0 + 0.1 * i, heading=(np.cos(th), np.sin(th), 0.02),
                                   wl=0.1 * (i % 3), wr=0.05 * (i % 5)))
    return out


def _run(arm, async_tail, steps, between=None, arm_wait_us=None):
    Z, hw, cm = hp.c3_scene()
    sts = _states(len(steps))
    eng = hp.engine_for(K, H, Z, hw, cm, sts[0])
    eng.set_option("arm", arm)
    if arm_wait_us is not None:
        eng.set_option("arm_wait_us", arm_wait_us)
    eng.set_async_tail(async_tail)
    outs = []
    for i, (st, s) in enumerate(zip(sts, steps)):
        eng.set_state(hp.state_for(st))
        o = eng.step("3d", s)
        if async_tail:
            o = eng.outputs()
        outs.append({k: np.array(o[k], copy=True) for k in KEYS})
        if between is not None:
            between(eng, i)
    info = eng.launch_info()
    eng.close()
    return outs, info


def _same(a, b):
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        for k in KEYS:
            assert np.array_equal(x[k], y[k]), f"step {i}: " + hp.mismatch_report(k, x[k], y[k])


@pytest.mark.parametrize("async_tail", [True, False], ids=["deferred-tail", "synchronous"])
def test_armed_steps_bitwise_closed_loop(async_tail):
    steps = list(range(12))
    ref, info0 = _run(0, async_tail, steps)
    got, info1 = _run(1, async_tail, steps)
    _same(got, ref)
    assert info0["armed_taken"] == 0
    # the first step runs the ordinary way (allocation), the second arms the third, ...; a slow
    # first call or two may find its gate expired (500 us), which is still the same result
    assert info1["armed_taken"] + info1["armed_expired"] >= len(steps) - 3, info1
    assert info1["armed_taken"] >= 3, info1


def test_armed_step_number_jump_and_interleaved_calls():
    steps = [0, 1, 2, 7, 8, 9, 10, 3, 4, 5]

    def between(eng, i):
        if i == 5:
            eng.costs()  # another call: cancels the armed step
    ref, _ = _run(0, True, steps, between)
    got, info = _run(1, True, steps, between)
    _same(got, ref)
    assert info["armed_cancelled"] >= 2, info  # the jumps 2 -> 7 and 10 -> 3, and the costs() call
    assert info["armed_taken"] >= 3, info


def test_armed_step_expired_gate():
    steps = list(range(6))

    def between(eng, i):
        if i in (1, 3):
            time.sleep(0.01)  # longer than the gate waits (50 us): it expires, the step runs anyway
    ref, _ = _run(0, True, steps, between)
    got, info = _run(1, True, steps, between, arm_wait_us=50)
    _same(got, ref)
    assert info["armed_expired"] >= 1, info


def test_sync_cancels_armed_step():
    """mppi_sync right after a step returns promptly (the armed step is cancelled, not waited out)."""
    Z, hw, cm = hp.c3_scene()
    st = _states(1)[0]
    eng = hp.engine_for(K, H, Z, hw, cm, st)
    eng.set_option("arm", 1)
    eng.set_option("arm_wait_us", 5_000_000)  # 5 s: waiting it out would show
    for s in range(3):
        eng.step("3d", s)
    t0 = time.perf_counter()
    eng.sync()
    dt = time.perf_counter() - t0
    info = eng.launch_info()
    eng.close()
    assert dt < 0.5, dt
    assert info["armed_cancelled"] >= 1, info
