"""CPU: the emitted control vector against the REFERENCE'S OWN float32 update arithmetic.

The engine (and the oracle's D2 tree, which it matches bit for bit) replaces the reference's
racy float32 softmax update with a fixed-order float64 tree.  These tests
measure how far that moves the emitted controls from what the reference itself computes:
``oracle.mppi_ref.reference_update_f32`` restates critics_warp.py:338-376 literally (exact
min, float32 weights, S summed in float32, each term (w*u)/S in float32 and accumulated in
float32), followed by the k=3.0, a=0.92 filter (MPPI_isaac.py:672-692).  Float atomics commit
in a hardware-dependent order, so it runs in index order and in 8 seeded permutations.

Tolerances (north_star: "<= 1e-5 relative on the emitted control vector"):
* at the reference's temperature (T = 0.3, config.yaml): every element within 1e-5 of every
  ordering (``rel_err``: |a-b| / max(|ref|, 1e-3) per element);
* at raised temperatures (many trajectories share the weight, the regime where summation
  order matters): the engine's u_opt is the exact weighted mean of the reference's own float32
  weights to < 1e-7, and max|a-b| / max(|ref|, 1e-3) <= 1e-5 against every ordering at C1/C2
  (whole-vector metric).  Per element the reference's orderings themselves spread up to 5e-5
  (an element much smaller than the vector's largest), so the per-element bound is stated against
  their envelope: each element of the engine lies within ENVELOPE_TOL = 2e-5 (relative, same
  scale) of [min, max] over the 9 orderings (measured worst 1.2e-5, C2 at T = 300; <= 2e-6 in
  the other cases).  Every tolerance and metric is the TOLS table below.
  At C3 with T = 1e5 (~15 500 effective samples) the reference's float32 recursive sums drift
  2e-5 from the exact mean: that is the reference's own rounding, measured in
  tests/test_gpu_headline.py and DESIGN.md §5.
"""
import numpy as np
import pytest

import helpers as hp
from oracle import dmath
from oracle import mppi_ref as R

F32 = np.float32
TOLS = {"T=0.3, per element vs every ordering": 1e-5,
        "raised T, whole vector vs every ordering": 1e-5,
        "raised T, per element outside the orderings' envelope": 2e-5}
TOL = TOLS["T=0.3, per element vs every ordering"]
ENVELOPE_TOL = TOLS["raised T, per element outside the orderings' envelope"]
KEYS = (("u1_opt", "u1_opt"), ("u2_opt", "u2_opt"), ("lin_vel", "v_opt"), ("ang_vel", "w_opt"))


def glob_err(a, b, floor=1e-3):
    """max|a-b| / max(max|b|, floor) over the whole vector."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(float(np.abs(b).max()), floor))


def exact_mean(cost, u, T):
    """sum_k w_k u_k / sum_k w_k in float64 with the reference's float32 weights."""
    c = np.asarray(cost, F32)
    w = dmath.dm_expf((-(c - c.min())) / F32(T)).astype(np.float64)
    return (w[:, None] * np.asarray(u, np.float64)).sum(0) / w.sum()


def _case(K, H, seed, T=0.3):
    sc = hp.oracle_scene(*hp.c3_scene())
    st = hp.oracle_state(wl=0.1 * seed, wr=0.15 * seed)
    p = R.Params(K=K, H=H, seed=seed, temperature=T)
    z = np.zeros(H, F32)
    ref = R.mppi_step(p, sc, st, z, z, 0)
    part = ref["parts"][0]
    return p, st, ref, part


def test_reference_update_is_literal():
    """The restatement against a scalar loop written straight from critics_warp.py:338-376."""
    rng = np.random.default_rng(3)
    K, H, T = 37, 5, F32(0.7)
    cost = (rng.random(K) * 3).astype(F32)
    u1 = rng.uniform(-1, 1, (K, H)).astype(F32)
    u2 = rng.uniform(-1, 1, (K, H)).astype(F32)
    order = rng.permutation(K)
    m = F32(np.inf)
    for k in range(K):                       # atomic_min
        m = min(m, cost[k])
    w = [F32(dmath.dm_expf(np.array([(-(cost[k] - m)) / T], F32))[0]) for k in range(K)]
    S = F32(0.0)
    for k in order:                          # atomic_add(weights_sum, w)
        S = F32(S + w[k])
    o1 = np.zeros(H, F32)
    o2 = np.zeros(H, F32)
    for k in order:                          # out[t] += w*u/S
        for t in range(H):
            o1[t] = F32(o1[t] + F32(F32(w[k] * u1[k, t]) / S))
            o2[t] = F32(o2[t] + F32(F32(w[k] * u2[k, t]) / S))
    a, b = R.reference_update_f32(cost, u1, u2, T, order, order)
    assert np.array_equal(a, o1) and np.array_equal(b, o2)


@pytest.mark.parametrize("K,H", [(256, 20), (4096, 50)])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_emitted_controls_vs_reference_f32(K, H, seed):
    """C1/C2 at the reference temperature: within 1e-5 per element of all 9 orderings."""
    p, st, ref, part = _case(K, H, seed)
    outs = R.reference_emitted_f32(p, st, part["cost"], part["u1"], part["u2"])
    for o in outs:
        for _, b in KEYS:
            assert hp.rel_err(ref[b], o[b]) <= TOL, (b, hp.rel_err(ref[b], o[b]))


@pytest.mark.parametrize("K,H", [(256, 20), (4096, 50)])
@pytest.mark.parametrize("T", [30.0, 300.0, 3000.0, 1e5])
def test_emitted_controls_vs_reference_f32_raised_temperature(K, H, T):
    """Many effective samples: D2 gives the exact weighted mean of the reference's float32 weights
    (< 1e-7), and the reference's float32 orderings sit within 1e-5 of it (whole-vector metric)."""
    p, st, ref, part = _case(K, H, 1, T)
    for k, u in (("u1_opt", part["u1"]), ("u2_opt", part["u2"])):
        assert glob_err(ref[k], exact_mean(part["cost"], u, T)) < 1e-7
    outs = R.reference_emitted_f32(p, st, part["cost"], part["u1"], part["u2"])
    for o in outs:
        for _, b in KEYS:
            assert glob_err(ref[b], o[b]) <= TOLS["raised T, whole vector vs every ordering"], (b, glob_err(ref[b], o[b]))
    for _, b in KEYS:  # per element: inside the envelope of the reference's own orderings
        assert outside_envelope(ref[b], [o[b] for o in outs]) <= ENVELOPE_TOL, (b, T)


def outside_envelope(e, outs, floor=1e-3):
    """Per element, how far e lies outside [min, max] over the orderings, relative to
    max(max |ordering|, floor) of that element."""
    O = np.stack([np.asarray(o, np.float64) for o in outs])
    e = np.asarray(e, np.float64)
    out = np.maximum(np.maximum(O.min(0) - e, e - O.max(0)), 0.0)
    return float((out / np.maximum(np.abs(O).max(0), floor)).max())
