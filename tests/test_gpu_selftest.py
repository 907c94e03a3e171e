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
