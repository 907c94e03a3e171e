"""Soak of the resident step server (not part of the product): C3 (K 65 536, H 100), N steps of
tests/test_gpu_server_soak.py's mixed cadence (back-to-back steps, host gaps around half the idle
limit and around it, get_outputs after ~30 % of the steps, a new state every step), then the same
calls as separate launches; prints the launch counters and the first mismatching step, if any.
usage: python profiles/ubench/soak.py [N]   (SOAK_RESIDENT: the server policy, "resident" 2 or 1; default 2)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402,F401
from test_gpu_server_soak import _schedule, run_schedule  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
gaps, read = _schedule(n, seed=11)
t0 = time.perf_counter()
mode = int(os.environ.get("SOAK_RESIDENT", "2"))
got, info = run_schedule(n, 100, {"resident": mode}, gaps, read)
t1 = time.perf_counter()
ref, _ = run_schedule(n, 100, {"resident": 0}, gaps, read)
t2 = time.perf_counter()
bad = next((i for i, (a, b) in enumerate(zip(got, ref)) if any(not np.array_equal(a[k], b[k]) for k in a)), None)
print(f"steps {n}: server run {t1 - t0:.1f} s, separate launches {t2 - t1:.1f} s")
print(f"resident {mode}, server launch info:", {k: info[k] for k in ("server_launches", "server_steps",
                                                  "server_failed_steps", "server_relaunches", "server_fallbacks",
                                                  "cadence_steps")})
print("outputs read:", int(read.sum()), " gaps (us) histogram:",
      dict(zip(*[x.tolist() for x in np.unique(gaps, return_counts=True)])))
print("first mismatch:", bad)
sys.exit(0 if bad is None and info["server_failed_steps"] == 0 else 1)
