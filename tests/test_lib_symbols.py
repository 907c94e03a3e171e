"""CPU: libmppi_hip.so loads and exports exactly the C-ABI that include/mppi.h declares.

No compute call is made (there is no GPU here); only mppi_abi_version() and
mppi_last_error(), which touch no device.
"""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mppi.h")
CSRC = os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd", "csrc")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(mppi_\w+)\s*\(", text, flags=re.M))


@pytest.fixture(scope="module")
def libpath():
    from mppi_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", CSRC, "-j8"], check=True)
    return _lib.LIB_PATH


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for must in ("mppi_create", "mppi_destroy", "mppi_set_dem", "mppi_set_costmap", "mppi_set_state",
                 "mppi_step", "mppi_step_partial", "mppi_step_finish", "mppi_last_error"):
        assert must in fns
    assert len(fns) >= 20


def test_library_exports_every_header_symbol(libpath):
    syms = exported(libpath)
    missing = header_functions() - syms
    assert not missing, f"declared in mppi.h but not exported: {sorted(missing)}"
    extra = {s for s in syms if s.startswith("mppi_")} - header_functions()
    assert not extra, f"exported but not declared: {sorted(extra)}"


def test_ctypes_prototypes_cover_header():
    from mppi_amd import _lib
    assert set(_lib._PROTOS) == header_functions()


def test_struct_layout_matches_header():
    """ctypes mirrors of mppi_params / mppi_state / mppi_outputs have the C sizes."""
    from mppi_amd import _lib
    # mppi_params: 2 x int64, 2 x int32, 23 x float, pad to 8, uint64
    assert ctypes.sizeof(_lib.MppiParams) == 8 + 8 + 4 + 4 + 23 * 4 + 4 + 8
    assert _lib.MppiParams.seed.offset % 8 == 0
    assert ctypes.sizeof(_lib.MppiState) == 11 * 4
    assert ctypes.sizeof(_lib.MppiOutputs) == 8 * ctypes.sizeof(ctypes.c_void_p)


def test_library_loads_and_reports_abi(libpath):
    from mppi_amd import _lib
    lib = _lib.load_library(libpath)
    assert lib.mppi_abi_version() == 1
    assert isinstance(lib.mppi_last_error(), bytes)


def test_missing_library_fails_loudly(tmp_path):
    from mppi_amd import _lib
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load_library(str(tmp_path / "libmppi_hip.so"))


def test_null_context_calls_are_refused(libpath):
    """Entry points called with a null context or out-of-range arguments return MPPI_EINVAL (-1) before
    touching any device (round-5 advisor: mppi_step(NULL) used to dereference the context)."""
    from mppi_amd import _lib
    lib = _lib.load_library(libpath)
    out = _lib.MppiOutputs()
    assert lib.mppi_step(None, 3, 0, ctypes.byref(out)) != 0
    assert b"null" in lib.mppi_last_error()
    u = (ctypes.c_float * 4)()
    assert lib.mppi_step_injected(None, 3, u, u, ctypes.byref(out)) != 0
    assert lib.mppi_set_option(None, b"resident", 1) != 0
    assert lib.mppi_group_step(None, 3, 0, ctypes.byref(out)) != 0
    assert lib.mppi_sync(None) != 0
    assert lib.mppi_debug_hold(0, None, 0, 1024, 10) != 0        # no workgroups
    assert lib.mppi_debug_hold(0, None, 1, 1 << 20, 10) != 0     # more LDS than a CU has
    assert lib.mppi_debug_hold(0, None, 1, 1024, 2_000_000) != 0  # longer than 1 s
