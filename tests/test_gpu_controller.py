"""GPU: the drop-in MPPI_Controller (MPPI_isaac.py surface) driven like MPPI_Controller.run, vs the oracle."""
import numpy as np
import pytest
import yaml

import helpers as hp
from oracle import mppi_ref as R

pytestmark = pytest.mark.gpu


def _config(K, H):
    from mppi_amd.controller import DEFAULT_CONFIG
    with open(DEFAULT_CONFIG) as f:
        c = yaml.safe_load(f)
    c["controller"]["number_of_trajectories"] = K
    c["controller"]["number_of_iterations"] = H
    return c


def test_controller_closed_loop_matches_oracle():
    """Five iterations of the run() loop body (MPPI_isaac.py:765-801): outputs bitwise equal to the oracle."""
    from mppi_amd.controller import MPPI_Controller, Robot, Surface
    K, H = 512, 24
    Z, hw, cm = hp.c3_scene()
    cfg = _config(K, H)
    surf = Surface.from_arrays(Z, cm, hw)
    robot = Robot(-60.0, -5.0, [1.0, 0.2, 0.0], cfg)
    ctl = MPPI_Controller(surf, robot, cfg, 65.0, 10.0, 2.2)
    ctl.warp_setup()

    p = R.Params(K=K, H=H, seed=42)
    sc = R.Scene(Z, hw, cm)
    x, y, hv = -60.0, -5.0, np.array([1.0, 0.2, 0.0]) / np.linalg.norm([1.0, 0.2, 0.0])
    wl = wr = 0.0
    s1 = s2 = 0.25
    u1n = np.zeros(H, np.float32)
    u2n = np.zeros(H, np.float32)
    for it in range(5):
        ctl.reset("controller")
        ctl.MPPI_step("3d")
        st = R.State(x=x, y=y, heading=hv, left_wheel_speed=wl, right_wheel_speed=wr, goal_x=65.0, goal_y=10.0,
                     std_dev_u1=s1, std_dev_u2=s2)
        ref = R.mppi_step(p, sc, st, u1n, u2n, it)
        u1n, u2n = ref["u1_opt"], ref["u2_opt"]
        np.testing.assert_array_equal(ctl.optimal_u1_wp.numpy(), ref["u1_opt"])
        np.testing.assert_array_equal(ctl.optimal_lin_vel_wp.numpy(), ref["v_opt"])
        np.testing.assert_array_equal(ctl.optimal_ang_vel_wp.numpy(), ref["w_opt"])
        np.testing.assert_array_equal(ctl.trajectories_sim.numpy(), ref["traj_sim"])
        np.testing.assert_array_equal(ctl.costs_wp.numpy(), ref["cost"])
        # the run() loop body
        traj = ctl.trajectories_sim.numpy()
        hs = ctl.heading_vectors_sim.numpy()
        robot.update_position(traj[0][0], traj[0][1], traj[0][2], hs[0])
        lin = ctl.optimal_lin_vel_wp.numpy()[0]
        ang = ctl.optimal_ang_vel_wp.numpy()[0]
        ctl.std_dev_u1 = np.maximum(0.4, 0.4 - ang * ang)
        ctl.std_dev_u2 = np.maximum(0.4, 0.4 + ang * ang)
        robot.left_wheel_speed = lin - ang * robot.radius / 2
        robot.right_wheel_speed = lin + ang * robot.radius / 2
        x, y, hv = traj[0][0], traj[0][1], hs[0]
        wl, wr = robot.left_wheel_speed, robot.right_wheel_speed
        s1, s2 = ctl.std_dev_u1, ctl.std_dev_u2
    # lazy full-rollout introspection (self.trajectories.numpy())
    tr = ctl.trajectories.numpy()
    assert tr.shape == (K * H, 3)
    np.testing.assert_array_equal(tr.reshape(K, H, 3), ref["parts"][0]["traj"])


def test_controller_step_alias_and_rebinding():
    """step()/get_action() aliases, costmap_wp.assign and Z_wp rebinding (visual_terrain_stack_full_terrain.py:563-567)."""
    import torch
    from mppi_amd.controller import MPPI_Controller, Robot, Surface
    K, H = 256, 16
    Z, hw, cm = hp.c3_scene()
    cfg = _config(K, H)
    robot = Robot(-60.0, -5.0, [1, 0, 0], cfg)
    robot.left_wheel_speed = robot.right_wheel_speed = 1.5     # moving: rollouts cross DEM cells
    ctl = MPPI_Controller(Surface.from_arrays(Z, cm, hw), robot, cfg, 65.0, 10.0, 0.0)
    ctl.warp_setup()
    a0 = ctl.step("3d")
    assert isinstance(a0, tuple) and len(a0) == 2 and a0 == ctl.get_action()
    # rebinding the DEM to a device tensor (zero copy) and reassigning the costmap change nothing here
    ctl.Z_wp = torch.from_numpy(Z).cuda()
    ctl.costmap_wp.assign(cm.ravel())
    ctl.reset("sim")
    assert not ctl.optimal_u1_wp.numpy().any()
    ctl.step_index = 0
    a1 = ctl.step("3d")
    assert a1 == a0
    # flattened warp-style upload of a different DEM: the engine now follows the new terrain
    Z2 = (Z * 3.0).astype(np.float32)
    ctl.Z_wp = Z2.ravel()
    ctl.reset("sim")
    ctl.step_index = 0
    a2 = ctl.step("3d")
    st = R.State(x=-60.0, y=-5.0, left_wheel_speed=1.5, right_wheel_speed=1.5, goal_x=65.0, goal_y=10.0)
    ref = R.mppi_step(R.Params(K=K, H=H, seed=42), R.Scene(Z2, hw, cm), st, np.zeros(H, np.float32),
                      np.zeros(H, np.float32), 0)
    np.testing.assert_array_equal(ctl.optimal_u1_wp.numpy(), ref["u1_opt"])
    np.testing.assert_array_equal(ctl.costs_wp.numpy(), ref["cost"])
    assert a2 == (float(ref["v_opt"][0]), float(ref["w_opt"][0]))
