"""Drop-in replacement of thesis_master/warp_implementation/MPPI_isaac.py (Surface, Robot, MPPI_Controller).

Same constructors, methods and attributes as the reference class surface used by
``MPPI_Controller.run`` (MPPI_isaac.py:755-806) and by the Isaac robot loop
(visual_terrain_stack_full_terrain.py:449-576); the step runs in the HIP engine
(libmppi_hip.so) through the C-ABI in include/mppi.h.  Warp arrays become
:class:`EngineArray` objects with the methods callers use (``.numpy()``,
``.assign()``, ``.zero_()``).

There is no CPU fallback: ``warp_setup()`` raises if the HIP library or a GPU
is missing.
"""
from __future__ import annotations

import os

import numpy as np
import yaml

from . import _lib, scene

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_CONFIG = os.path.join(_HERE, "config.yaml")


def _load_config(config):
    """YAML path or mapping -> dict (MPPI_isaac.py:383-384, :406-407 use yaml.safe_load)."""
    if isinstance(config, dict):
        return config
    with open(config, "r") as f:
        return yaml.safe_load(f)


class EngineArray:
    """Host-side stand-in for a wp.array of the reference controller.

    ``numpy()`` returns a copy of the current values (fetched from the engine
    when needed); ``assign(values)`` uploads; ``zero_()`` zeroes.
    """

    def __init__(self, getter, setter=None, name=""):
        self._get = getter
        self._set = setter
        self.name = name

    def numpy(self):
        return np.array(self._get(), copy=True)

    def assign(self, values):
        if self._set is None:
            raise AttributeError(f"{self.name} is read-only")
        self._set(np.asarray(values))

    def zero_(self):
        self.assign(np.zeros_like(self.numpy()))

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def __len__(self):
        return len(self._get())

    @property
    def shape(self):
        return np.shape(self._get())

    def __repr__(self):
        return f"EngineArray({self.name}, shape={self.shape})"


# =====================================================================  Surface
class Surface:
    """Scene container (MPPI_isaac.py:259-378): DEM Z, costmap and their grid geometry."""

    def __init__(self, which_map, filename, which_costmap, costmap_file, grid_size, half_width, origin,
                 bumps, radius_robot, obstacles=[]):
        self.grid_size = grid_size
        self.r_robot = radius_robot
        self.half_width = half_width
        self.resolution = 2 * self.half_width / self.grid_size            # :265
        x = np.linspace(-self.half_width, self.half_width, grid_size)
        self.X, self.Y = np.meshgrid(x, x)
        self.costmap_size = int(self.grid_size / 8)                       # :271
        self.costmap_resolution = 2 * self.half_width / self.costmap_size  # :272
        xc = np.linspace(-self.half_width, self.half_width, self.costmap_size)
        self.X_costmap, self.Y_costmap = np.meshgrid(xc, xc)
        self.Z = np.zeros_like(self.X)
        self.costmap = None
        self.obstacles = obstacles
        if which_map == "manual":
            self.X, self.Y, self.Z = self.create_surface(bumps)
        if which_map == "imported":
            self.X, self.Y, self.Z = self.import_surface(filename, 1000, 2500, bumps)
        if which_costmap == "manual":
            self.costmap = self.create_obstacles_costmap(obstacles, origin)
        if which_map == "imported" or which_costmap == "imported":
            self.costmap = self.import_obstacles_costmap(costmap_file)

    @classmethod
    def from_arrays(cls, Z, costmap, half_width, radius_robot=1.2):
        """Scene from in-memory arrays (DEM grid_size x grid_size, costmap size x size)."""
        s = cls.__new__(cls)
        Z = np.asarray(Z)
        s.grid_size = Z.shape[1]
        s.r_robot = radius_robot
        s.half_width = half_width
        s.resolution = 2 * half_width / s.grid_size
        s.Z = Z
        s.costmap = np.asarray(costmap)
        s.costmap_size = s.costmap.shape[1]
        s.costmap_resolution = 2 * half_width / s.costmap_size
        s.obstacles = []
        x = np.linspace(-half_width, half_width, s.grid_size)
        s.X, s.Y = np.meshgrid(x, x)
        xc = np.linspace(-half_width, half_width, s.costmap_size)
        s.X_costmap, s.Y_costmap = np.meshgrid(xc, xc)
        return s

    def import_surface(self, filename, start_index, end_index, bumps):
        """MPPI_isaac.py:299-305 (np.load; pickles are never loaded)."""
        x = np.linspace(-self.half_width, self.half_width, end_index - start_index)
        X, Y = np.meshgrid(x, x)
        Z = np.load(filename, allow_pickle=False)
        return X, Y, Z

    def create_surface(self, bumps):
        """MPPI_isaac.py:307-356 (crater field)."""
        Z = scene.crater_dem(self.grid_size, self.half_width, bumps).astype(np.float64)
        x = np.linspace(-self.half_width, self.half_width, self.grid_size)
        X, Y = np.meshgrid(x, x)
        return X, Y, Z

    def import_obstacles_costmap(self, costmap_file):
        return np.load(costmap_file, allow_pickle=False)

    # device the HIP costmap builder runs on (the reference's Warp arrays live on "cuda" = device 0)
    device = 0
    # distance metric of the costmap builder: "chamfer" = cv2.distanceTransform(DIST_L2, 5) (reference)
    costmap_metric = "chamfer"

    def create_obstacles_costmap(self, obstacles, origin):
        """MPPI_isaac.py:361-378 on the GPU (csrc/mppi_costmap.hip): disc raster, cv2.distanceTransform
        (DIST_L2, 5) as OpenCV's published 5x5 chamfer, min-max normalise, (1 - d)**20; returns the
        ndarray (``costmap_metric = "exact"`` selects the exact EDT instead)."""
        from . import _lib
        b = getattr(self, "_builder", None)
        if b is None:
            b = self._builder = _lib.CostmapBuilder(self.device)
        self.obstacles = obstacles
        return b.build(obstacles, origin, self.costmap_size, self.half_width, self.r_robot, power=20,
                       metric=self.costmap_metric)


# =====================================================================  Robot
class Robot:
    """MPPI_isaac.py:381-400."""

    def __init__(self, x, y, heading_vector, config_file):
        config = _load_config(config_file)
        self.x = [x]
        self.y = [y]
        self.z = [0]
        self.lin_vel = []
        self.ang_vel = []
        self.heading_vector = np.array(heading_vector) / np.linalg.norm(heading_vector)
        self.radius = config["frame_work"]["robot_radius"]
        self.left_wheel_speed = 0.0
        self.right_wheel_speed = 0.0

    def update_position(self, new_x, new_y, new_z, new_heading):
        self.x.append(new_x)
        self.y.append(new_y)
        self.z.append(new_z)
        self.heading_vector = new_heading


# =====================================================================  MPPI_Controller
class MPPI_Controller:
    """MPPI_isaac.py:402-806 on the MI355X engine.

    Extra (optional) config section ``engine:`` — ``seed`` (Philox key, default
    42 as default_rng(42) at :409), ``device`` (HIP device, default 0),
    ``max_loops`` (run(), default 3500 as :763), ``async_tail``, ``resident`` (the resident
    step server: true / 1 for back-to-back calls (default), 2 always, false / 0 never;
    mppi_set_option "resident"; env MPPI_RESIDENT wins when set),
    ``resident_idle_us`` (how long an idle server stays resident, 200: DESIGN.md §3.5).
    """

    def __init__(self, surface, robot, config_path, goal_x, goal_y, goal_orientation):
        config = _load_config(config_path)
        self.config = config
        self.robot = robot
        self.surface = surface
        self.goal_x = goal_x
        self.goal_y = goal_y
        self.goal_orientation = goal_orientation
        self.loop = 0
        c, vel, inp = config["controller"], config["velocities"], config["inputs"]
        self.number_of_iterations = c["number_of_iterations"]
        self.dt = c["dt"]
        self.number_of_trajectories = c["number_of_trajectories"]
        self.initial_linear_velocity = vel["initial_linear_velocity"]
        self.std_dev_u1 = inp["std_dev_u1"]
        self.min_u1 = inp["min_u1"]
        self.max_u1 = inp["max_u1"]
        self.std_dev_u2 = inp["std_dev_u2"]
        self.min_u2 = inp["min_u2"]
        self.max_u2 = inp["max_u2"]
        self.initial_angular_velocity = vel["initial_angular_velocity"]
        self.v_min_linear = vel["min_linear_velocity"]
        self.v_max_linear = vel["max_linear_velocity"]
        self.v_min_angular = vel["min_angular_velocity"]
        self.v_max_angular = vel["max_angular_velocity"]
        self.temperature = config["cost_evaluation"]["temperature"]
        self.horizon = self.dt * self.v_max_linear * self.number_of_iterations   # :440
        eng = config.get("engine", {}) or {}
        self.seed = int(eng.get("seed", 42))
        self.device = int(eng.get("device", 0))
        self.max_loops = int(eng.get("max_loops", 3500))
        # deferred optimal rollout: MPPI_step returns with the controls and row 0 of the
        # *_sim arrays; the other rows are fetched on first access (bitwise identical)
        self.async_tail = bool(eng.get("async_tail", True))
        # the resident step server and its idle limit (mppi_set_option); the environment's
        # MPPI_RESIDENT, when set, takes precedence over the config (profiling runs turn it off)
        self.resident = None if os.environ.get("MPPI_RESIDENT") is not None or "resident" not in eng \
            else int(eng["resident"])  # (true / false, or 0 / 1 / 2: mppi_set_option "resident")
        self.resident_idle_us = eng.get("resident_idle_us")
        self.step_index = 0          # Philox step counter (replaces rng.integers at :517)
        self.engine = None
        self._out = None

    # ------------------------------------------------------------ setup
    def _params(self):
        return _lib.make_params(
            self.number_of_trajectories, self.number_of_iterations, dt=self.dt,
            robot_radius=self.robot.radius, min_u1=self.min_u1, max_u1=self.max_u1,
            min_u2=self.min_u2, max_u2=self.max_u2, v_min_linear=self.v_min_linear,
            v_max_linear=self.v_max_linear, v_min_angular=self.v_min_angular,
            v_max_angular=self.v_max_angular, temperature=self.temperature, horizon=self.horizon,
            seed=self.seed)

    def warp_setup(self):
        """MPPI_isaac.py:442-487: allocate the engine and upload DEM + costmap."""
        if self.engine is not None:
            self.engine.close()
        self.engine = _lib.Engine(self._params(), self.device)
        self.engine.set_async_tail(self.async_tail)
        if self.resident is not None:
            self.engine.set_option("resident", self.resident)
        if self.resident_idle_us is not None:
            self.engine.set_option("resident_idle_us", int(self.resident_idle_us))
        self._tail_fresh = True
        self._upload_dem(self.surface.Z)
        self._upload_costmap(self.surface.costmap)
        H, K = self.number_of_iterations, self.number_of_trajectories
        z3 = np.zeros((H, 3), np.float32)
        self._out = dict(u1_opt=np.zeros(H, np.float32), u2_opt=np.zeros(H, np.float32),
                         lin_vel=np.full(H, self.initial_linear_velocity, np.float32),
                         ang_vel=np.full(H, self.initial_angular_velocity, np.float32),
                         traj_sim=z3, heading_sim=z3.copy(), left_wheel_sim=z3.copy(),
                         right_wheel_sim=z3.copy())
        self._dump = None
        o = self._out
        self.optimal_u1_wp = EngineArray(lambda: self.engine.get_nominal()[0],
                                         lambda v: self._set_nominal(v, None), "optimal_u1_wp")
        self.optimal_u2_wp = EngineArray(lambda: self.engine.get_nominal()[1],
                                         lambda v: self._set_nominal(None, v), "optimal_u2_wp")
        self.optimal_lin_vel_wp = EngineArray(lambda: self._out["lin_vel"], name="optimal_lin_vel_wp")
        self.optimal_ang_vel_wp = EngineArray(lambda: self._out["ang_vel"], name="optimal_ang_vel_wp")
        self.trajectories_sim = EngineArray(lambda: self._sim("traj_sim"), name="trajectories_sim")
        self.heading_vectors_sim = EngineArray(lambda: self._sim("heading_sim"), name="heading_vectors_sim")
        self.left_wheel_pos_sim = EngineArray(lambda: self._sim("left_wheel_sim"), name="left_wheel_pos_sim")
        self.right_wheel_pos_sim = EngineArray(lambda: self._sim("right_wheel_sim"), name="right_wheel_pos_sim")
        self.costs_wp = EngineArray(self._costs, name="costs_wp")
        self.weights_wp = EngineArray(self._weights, name="weights_wp")
        self.costmap_wp = EngineArray(lambda: np.asarray(self.surface.costmap, np.float32).ravel(),
                                      self._assign_costmap, "costmap_wp")
        for name, key, shape3 in (("trajectories", "traj", True), ("heading_vectors", "hv", True),
                                  ("left_wheel_pos", "lw", True), ("right_wheel_pos", "rw", True),
                                  ("linear_velocities", "v", False), ("angular_velocities", "w", False),
                                  ("u1", "u1", False), ("u2", "u2", False)):
            setattr(self, name, EngineArray(self._dumped(key, K * H, shape3), name=name))
        self.previous_heading_vector = np.asarray(self.robot.heading_vector, np.float32)
        del o

    # ------------------------------------------------------------ device-array plumbing
    def _upload_dem(self, Z):
        """Z_wp binding (visual_terrain_stack_full_terrain.py:567: ``controller_3d.Z_wp = DEM_warp``).

        Device arrays are bound zero copy: anything exposing ``__cuda_array_interface__`` (a Warp
        array such as the terrain manager's ``dem_wp``, geometry_clipmaps.py:300/332), a CUDA
        ``torch.Tensor``, or a ``__dlpack__`` producer on the GPU.  They must be float32 and
        C-contiguous (refused otherwise: a silent copy would stop following the caller's buffer),
        1-D of n*n cells (the reference's flat dem_wp) or 2-D (rows, cols).  Host arrays (ndarray,
        ``.numpy()``/``__array__`` objects) are uploaded.  After an in-place write of a bound
        device DEM call :meth:`dem_updated` (or bind it again).
        """
        hw = self.surface.half_width
        dev = _device_dem(Z)
        if dev is not None:
            ptr, rows, cols, keep = dev
            self.engine.set_dem_device(ptr, rows, cols, hw, keepalive=keep)
            return
        if hasattr(Z, "numpy") and not isinstance(Z, np.ndarray):
            Z = Z.numpy()
        Z = np.asarray(Z, np.float32)
        if Z.ndim == 1:
            n = int(round(np.sqrt(Z.size)))
            Z = Z.reshape(n, n)
        self.engine.set_dem(Z, hw)

    def dem_updated(self):
        """The bound device DEM was written in place (geometry_clipmaps.py:293 ``dem_wp.assign``):
        rebuild the per-cell normal table the rollout reads (the reference's kernels read the live
        heights at every step)."""
        self.engine.dem_updated()

    def _upload_costmap(self, cm):
        cm = np.asarray(cm, np.float32)
        if cm.ndim == 1:
            n = int(round(np.sqrt(cm.size)))
            cm = cm.reshape(n, n)
        self.engine.set_costmap(cm, self.surface.half_width, self.surface.costmap_resolution)

    def _assign_costmap(self, flat):
        self.surface.costmap = np.asarray(flat, np.float32).reshape(
            self.surface.costmap_size, self.surface.costmap_size)
        self._upload_costmap(self.surface.costmap)

    def rebuild_costmap(self, obstacles, origin):
        """surface.costmap = surface.create_obstacles_costmap(rocks, origin) + costmap_wp.assign(...)
        (visual_terrain_stack_full_terrain.py:561-563) in one device pass: the map is built in the
        engine's own costmap buffer (no upload) and copied back once for surface.costmap."""
        if self.engine is None:
            raise RuntimeError("call warp_setup() first")
        s = self.surface
        s.obstacles = obstacles
        s.costmap = self.engine.build_costmap(obstacles, origin, s.costmap_size, s.half_width, s.r_robot, 20,
                                              metric=getattr(s, "costmap_metric", "chamfer"))
        return s.costmap

    @property
    def Z_wp(self):
        return EngineArray(lambda: np.asarray(self.surface.Z, np.float32).ravel(), self._upload_dem, "Z_wp")

    @Z_wp.setter
    def Z_wp(self, value):
        """controller.Z_wp = DEM_warp (visual_terrain_stack_full_terrain.py:567)."""
        self._upload_dem(value)

    @property
    def goal(self):
        return (self.goal_x, self.goal_y)

    @goal.setter
    def goal(self, value):
        self.goal_x, self.goal_y = float(value[0]), float(value[1])

    def _set_nominal(self, u1, u2):
        c1, c2 = self.engine.get_nominal()
        self.engine.set_nominal(c1 if u1 is None else u1, c2 if u2 is None else u2)

    def _sim(self, key):
        """Optimal-rollout arrays; waits for the deferred rollout on first access after a step."""
        if not self._tail_fresh:
            self._out = self.engine.outputs()
            self._tail_fresh = True
        return self._out[key]

    def _costs(self):
        return self.engine.costs()

    def _weights(self):
        """exp(-(c - min)/T) of the last step (critics_warp.py:338-347), for inspection."""
        c = self.engine.costs().astype(np.float64)
        return np.exp(-(c - c.min()) / self.temperature).astype(np.float32)

    def _dumped(self, key, n, vec3):
        def get():
            if self._dump is None:
                self._dump = self.engine.dump()
            a = self._dump[key]
            return a.reshape(n, 3) if vec3 else a.reshape(n)
        return get

    # ------------------------------------------------------------ the step
    def _state(self):
        return _lib.make_state(self.robot.x[-1], self.robot.y[-1], self.robot.heading_vector,
                               self.robot.left_wheel_speed, self.robot.right_wheel_speed,
                               self.goal_x, self.goal_y, self.std_dev_u1, self.std_dev_u2)

    def reset(self, controller_or_sim):
        """MPPI_isaac.py:489-503.  "controller": re-read the robot pose; "sim": zero the nominal sequence."""
        if self.engine is None:
            raise RuntimeError("call warp_setup() first")
        self.previous_heading_vector = np.asarray(
            self.robot.heading_vector / np.linalg.norm(self.robot.heading_vector), np.float32)
        if controller_or_sim == "controller":
            self.engine.set_state(self._state())
        else:
            H = self.number_of_iterations
            self.engine.set_nominal(np.zeros(H, np.float32), np.zeros(H, np.float32))

    def MPPI_step(self, proj):
        """MPPI_isaac.py:505-720: one sample/rollout/cost/update step; outputs land in host memory."""
        if self.engine is None:
            raise RuntimeError("call warp_setup() first")
        self.engine.set_state(self._state())
        self._out = self.engine.step(proj, self.step_index)
        self._tail_fresh = not self.async_tail
        self._dump = None
        self.step_index += 1

    # aliases requested by the drop-in contract
    def step(self, proj="3d"):
        """reset("controller") + MPPI_step(proj); returns (v0, omega0)."""
        self.reset("controller")
        self.MPPI_step(proj)
        return self.get_action()

    def get_action(self):
        """First optimal (linear, angular) velocity, as the Isaac loop reads it (:471-472)."""
        return float(self._out["lin_vel"][0]), float(self._out["ang_vel"][0])

    def run(self, proj):
        """Standalone closed loop (MPPI_isaac.py:755-806)."""
        self.warp_setup()
        while ((abs(self.robot.x[-1] - self.goal_x) > 0.5 or abs(self.robot.y[-1] - self.goal_y) > 0.5)
               and self.loop < self.max_loops):
            self.reset("controller")
            self.MPPI_step(proj=proj)
            # row 0 of the optimal rollout is returned with the step itself
            traj = self._out["traj_sim"]
            hv = self._out["heading_sim"]
            self.robot.update_position(traj[0][0], traj[0][1], traj[0][2], hv[0])
            lin_vel = self.optimal_lin_vel_wp.numpy()[0]
            ang_vel = self.optimal_ang_vel_wp.numpy()[0]
            self.std_dev_u1 = np.maximum(0.4, 0.4 - ang_vel * ang_vel)
            self.std_dev_u2 = np.maximum(0.4, 0.4 + ang_vel * ang_vel)
            self.robot.lin_vel.append(lin_vel)
            self.robot.ang_vel.append(ang_vel)
            self.robot.left_wheel_speed = lin_vel - ang_vel * self.robot.radius / 2
            self.robot.right_wheel_speed = lin_vel + ang_vel * self.robot.radius / 2
            self.loop += 1
        print("Number of loops:", self.loop)


def _grid_shape(shape):
    """(rows, cols) of a DEM buffer: 2-D as given, 1-D of n*n cells as n x n."""
    if len(shape) == 2:
        return int(shape[0]), int(shape[1])
    if len(shape) == 1:
        n = int(round(np.sqrt(shape[0])))
        if n * n != shape[0]:
            raise ValueError(f"1-D DEM of {shape[0]} cells is not square")
        return n, n
    raise ValueError(f"DEM must be 1-D (n*n) or 2-D, got shape {tuple(shape)}")


def _device_dem(Z):
    """(device pointer, rows, cols, keepalive) for a GPU-resident float32 C-contiguous DEM, None for a
    host array; raises for a device array that would need a copy."""
    cai = getattr(Z, "__cuda_array_interface__", None)
    if cai is not None:
        shape = tuple(cai["shape"])
        if cai.get("typestr") not in ("<f4", "=f4", "f4"):
            raise ValueError(f"device DEM must be float32, got typestr {cai.get('typestr')!r}")
        strides = cai.get("strides")
        if strides is not None and tuple(strides) != tuple(
                4 * int(np.prod(shape[i + 1:])) for i in range(len(shape))):
            raise ValueError(f"device DEM must be C-contiguous, got strides {strides}")
        rows, cols = _grid_shape(shape)
        return int(cai["data"][0]), rows, cols, Z
    try:
        import torch
    except ImportError:
        torch = None
    if torch is not None and not isinstance(Z, torch.Tensor) and hasattr(Z, "__dlpack__"):
        dev = Z.__dlpack_device__()[0] if hasattr(Z, "__dlpack_device__") else None
        if dev in (2, 10):  # kDLCUDA, kDLROCM: a device producer, viewed as a tensor (no copy)
            Z = torch.from_dlpack(Z)
    if torch is not None and isinstance(Z, torch.Tensor) and Z.is_cuda:
        if Z.dtype != torch.float32:
            raise ValueError(f"device DEM must be float32, got {Z.dtype}")
        if not Z.is_contiguous():
            raise ValueError("device DEM must be contiguous (bind a contiguous buffer: a copy would not "
                             "follow the caller's updates)")
        rows, cols = _grid_shape(tuple(Z.shape))
        return Z.data_ptr(), rows, cols, Z
    return None
