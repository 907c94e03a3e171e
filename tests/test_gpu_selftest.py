"""Device self-tests of the exact-arithmetic fast paths (bitwise vs IEEE operators)."""
import pytest

import helpers as hp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("what,name", [(0, "division"), (1, "sqrt"), (2, "lean normalisation"),
                                       (3, "lean normalisation, dominant component")])
def test_fast_paths_bitwise(what, name):
    st = hp.oracle_state()
    Z, hw, cm = hp.c3_scene()
    eng = hp.engine_for(64, 4, Z, hw, cm, st)
    for seed in (1, 2, 3):
        bad = eng.selftest(what, n=1 << 24, seed=seed)
        assert bad == 0, f"{name}: {bad} of 2^24 results differ from IEEE"


def test_one_correction_quotient_exhaustive_slice():
    """The chain's quotient with ONE residual correction (lean_div_s) equals IEEE a / b for every
    significand of a and 3 x 32768 divisor significands (2^38 pairs per seed); all 2^46 pairs ran in
    profiles/ubench/div1_check.hip (profiles/r04_div1_check.txt)."""
    st = hp.oracle_state()
    Z, hw, cm = hp.c3_scene()
    eng = hp.engine_for(64, 4, Z, hw, cm, st)
    for seed in (0, 1, 4093):
        bad = eng.selftest(4, n=1 << 38, seed=seed)
        assert bad == 0, f"{bad} of 2^38 quotients differ from IEEE"


def test_noise_radius_sqrt_exhaustive():
    """The noise kernels' square root of -2 log(u) (mppi_detmath.h sqrt_bm: v_sqrt_f32 and the
    neighbour residual test) equals IEEE sqrtf for -0, +0 and every float in [2^-24, 34], the range
    of the argument (u in [2^-24, 1])."""
    st = hp.oracle_state()
    Z, hw, cm = hp.c3_scene()
    eng = hp.engine_for(64, 4, Z, hw, cm, st)
    n = 2 + (0x42080000 - 0x33800000) + 1
    assert eng.selftest(5, n=n, seed=0) == 0
