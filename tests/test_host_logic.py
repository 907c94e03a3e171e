"""CPU: host-side logic of the drop-in (config parsing, scene geometry, parameter packing)."""
import os

import numpy as np
import pytest
import yaml

from mppi_amd import _lib, scene
from mppi_amd.controller import DEFAULT_CONFIG, EngineArray, MPPI_Controller, Robot, Surface
from oracle import mppi_ref as R


def _cfg(**over):
    with open(DEFAULT_CONFIG) as f:
        c = yaml.safe_load(f)
    for k, v in over.items():
        sec, key = k.split(".")
        c[sec][key] = v
    return c


def test_config_matches_reference_defaults():
    """config.yaml keys/values of thesis_master/warp_implementation/config.yaml."""
    c = _cfg()
    assert c["frame_work"]["robot_radius"] == 1.2
    assert c["controller"] == {"number_of_iterations": 100, "dt": 0.045, "number_of_trajectories": 1000}
    assert c["cost_evaluation"]["temperature"] == 0.3
    assert c["inputs"]["std_dev_u1"] == 0.25 and c["inputs"]["max_u2"] == 1


def test_surface_geometry_manual():
    """Surface (MPPI_isaac.py:259-378): resolution, costmap size/resolution, crater DEM, obstacle costmap."""
    s = Surface("manual", None, "none", None, 160, 8.0, (0.0, 0.0), scene.BUMPS_9[:2], 1.2)
    assert s.resolution == pytest.approx(0.1)
    assert s.costmap_size == 20 and s.costmap_resolution == pytest.approx(0.8)
    assert s.Z.shape == (160, 160)
    assert np.isfinite(s.Z).all()
    # the "manual" costmap is built by the HIP builder (tests/test_gpu_costmap.py)


def test_surface_from_arrays_and_import(tmp_path):
    Z = np.random.default_rng(0).normal(size=(64, 64)).astype(np.float32)
    cm = np.random.default_rng(1).uniform(size=(8, 8)).astype(np.float32)
    s = Surface.from_arrays(Z, cm, 3.2)
    assert s.resolution == pytest.approx(0.1) and s.costmap_size == 8
    np.save(tmp_path / "z.npy", Z)
    np.save(tmp_path / "c.npy", cm)
    s2 = Surface("imported", str(tmp_path / "z.npy"), "imported", str(tmp_path / "c.npy"), 64, 3.2,
                 (0, 0), [], 1.2)
    assert np.array_equal(s2.Z, Z) and np.array_equal(s2.costmap, cm)


def test_robot_contract():
    r = Robot(1.0, 2.0, [3.0, 4.0, 0.0], DEFAULT_CONFIG)
    assert r.x == [1.0] and r.y == [2.0] and r.z == [0]
    assert np.allclose(r.heading_vector, [0.6, 0.8, 0.0])
    assert r.radius == 1.2 and r.left_wheel_speed == 0.0 and r.right_wheel_speed == 0.0
    r.update_position(1.5, 2.5, 0.1, np.array([1.0, 0.0, 0.0]))
    assert r.x[-1] == 1.5 and r.y[-1] == 2.5 and r.z[-1] == 0.1


def test_controller_reads_config():
    s = Surface.from_arrays(np.zeros((32, 32), np.float32), np.zeros((4, 4), np.float32), 1.6)
    r = Robot(0.0, 0.0, [1.0, 0.0, 0.0], DEFAULT_CONFIG)
    c = MPPI_Controller(s, r, _cfg(**{"controller.number_of_trajectories": 512}), 5.0, 1.0, 0.3)
    assert c.number_of_trajectories == 512 and c.number_of_iterations == 100
    assert c.horizon == pytest.approx(0.045 * 2.0 * 100)
    assert c.goal == (5.0, 1.0)
    c.goal = (2.0, -1.0)
    assert (c.goal_x, c.goal_y) == (2.0, -1.0)
    p = c._params()
    assert p.num_trajectories == 512 and p.seed == 42
    assert np.float32(p.temperature) == np.float32(0.3)


def test_params_match_oracle_float32():
    """make_params rounds like the oracle's Params (Warp receives float32 kernel args)."""
    p = _lib.make_params(1000, 100)
    o = R.Params(K=1000, H=100)
    for name in ("dt", "robot_radius", "temperature", "filter_k", "filter_a", "opt_filter_k",
                 "opt_filter_a", "wheel_offset", "w_path", "w_slope", "w_speed", "w_obstacle",
                 "collision_threshold", "collision_penalty"):
        assert np.float32(getattr(p, name)) == o.f(name), name
    assert np.float32(p.horizon) == o.horizon_f32()


def test_state_heading_normalised_like_oracle():
    h = (0.3, -2.0, 0.7)
    s = _lib.make_state(1.0, 2.0, h)
    st = R.State(x=1.0, y=2.0, heading=np.array(h))
    assert np.array_equal(np.array(s.heading[:], np.float32), st.heading_f32())


def test_engine_array_semantics():
    store = {"v": np.arange(6, dtype=np.float32)}
    a = EngineArray(lambda: store["v"], lambda v: store.__setitem__("v", v.astype(np.float32)), "x")
    got = a.numpy()
    got[0] = 99
    assert store["v"][0] == 0          # numpy() is a copy
    a.assign(np.ones(6))
    assert np.array_equal(a.numpy(), np.ones(6))
    a.zero_()
    assert not a.numpy().any()
    assert len(a) == 6 and a.shape == (6,)
    ro = EngineArray(lambda: store["v"], name="ro")
    with pytest.raises(AttributeError):
        ro.assign(np.zeros(6))


@pytest.mark.skipif(__import__("torch").cuda.device_count() > 0, reason="checks the no-GPU failure mode")
def test_warp_setup_fails_loudly_without_gpu():
    """No CPU fallback: allocating the engine on a machine without a HIP device raises."""
    s = Surface.from_arrays(np.zeros((32, 32), np.float32), np.zeros((4, 4), np.float32), 1.6)
    r = Robot(0.0, 0.0, [1.0, 0.0, 0.0], DEFAULT_CONFIG)
    c = MPPI_Controller(s, r, DEFAULT_CONFIG, 5.0, 1.0, 0.3)
    with pytest.raises(RuntimeError):
        c.warp_setup()
    with pytest.raises(RuntimeError):
        c.MPPI_step("3d")


def test_scene_recipes_deterministic():
    a = scene.random_obstacles()
    b = scene.random_obstacles()
    assert a == b and len(a) == 750
    Z = scene.crater_dem(300, 15.0)
    assert Z.dtype == np.float32 and Z.shape == (300, 300)
    assert np.array_equal(Z, scene.crater_dem(300, 15.0))
