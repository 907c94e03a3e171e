"""CPU: the C-ABI group's member threads (mppi_group_step with n > 1 runs members 1..n-1 on threads
of their own), through mppi_group_selftest: the same handshake (generation counter,
pending count, spin-then-sleep) with host-only member steps, no GPU.  A member whose step fails must
not leave the others (or the caller) waiting, the failure must name that member, and later steps
must still run."""
import ctypes as C
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd"))


def _selftest(n, fail_member, steps):
    from mppi_amd import _lib
    lib = _lib.load_library()
    info = (C.c_int64 * 5)()
    assert lib.mppi_group_selftest(n, fail_member, steps, info) == 0, lib.mppi_last_error()
    return dict(zip(("returned", "failed", "named", "workers", "spin_us"), [int(x) for x in info]))


@pytest.mark.timeout(60)
@pytest.mark.parametrize("n,fail_member", [(2, 1), (4, 0), (8, 5), (8, 7)])
def test_failing_member_does_not_hang(n, fail_member):
    r = _selftest(n, fail_member, 50)
    assert r == {"returned": 50, "failed": 50, "named": 50, "workers": n - 1, "spin_us": r["spin_us"]}, r


@pytest.mark.timeout(60)
def test_no_failure_and_spin_policy():
    """No member fails: every step succeeds.  Workers spin only while the caller and the workers can
    each hold a granted CPU (affinity / cgroup quota), else they sleep at once."""
    r = _selftest(8, 8, 200)
    assert r["returned"] == 200 and r["failed"] == 0 and r["workers"] == 7, r
    cpus = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            cpus = min(cpus, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    assert r["spin_us"] == (200 if 8 < cpus else 0), (r, cpus)
    big = _selftest(max(cpus + 1, 2), cpus + 1, 20)
    assert big["failed"] == 0 and big["spin_us"] == 0, big
