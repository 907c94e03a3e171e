"""CPU: the packed Box-Muller pair the noise kernels run (mppi_detmath.h noise_block_pk) is bit-identical
to the scalar noise_block (and so to oracle.dmath.noise_block, pinned in test_oracle_golden.py).

Compiles tests/native/noise_pack_check.cpp for the host with the library's float flags
(-ffp-contract=off) and runs it over 2M random Philox blocks, every edge of the 24-bit uniforms and
the sincos octant boundaries.  Packed FP32 is IEEE per half on gfx950 as on the host.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle import dmath

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd", "csrc")


def _compiler():
    for c in ("/opt/rocm/llvm/bin/clang++", shutil.which("clang++") or ""):
        if c and os.path.exists(c):
            return c
    return None


def test_packed_box_muller_bit_identical(tmp_path):
    cxx = _compiler()
    if cxx is None:
        pytest.skip("no clang++")
    exe = str(tmp_path / "noise_pack_check")
    flags = ["-O2", "-std=c++17", "-ffp-contract=off", f"-I{CSRC}", f"-I{os.path.join(ROOT, 'include')}",
             "-D__HIP_PLATFORM_AMD__", "-isystem", "/opt/rocm/include"]
    cmd = [cxx, *flags, "-x", "hip", "--offload-arch=gfx950", "--cuda-host-only",
           os.path.join(HERE, "native", "noise_pack_check.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    out = subprocess.run([exe, "2000000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "0 mismatches" in out.stdout


def test_oracle_noise_block_matches_scalar_box_muller():
    """The oracle's noise_block is the scalar sequence the packed one is checked against (a spot
    check; Random123 / rocRAND vectors pin Philox in test_oracle_golden.py)."""
    z = dmath.noise_block(7, 3, np.arange(4, dtype=np.int64))
    assert all(np.all(np.isfinite(v)) for v in z)
