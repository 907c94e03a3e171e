"""ctypes binding of libmppi_hip.so (include/mppi.h).

The product path has no fallback: if the HIP library is missing or no GPU is
visible, every entry point raises.  Build it with ``python -c "import
__graft_entry__ as g; g.build()"`` (or ``make -C husky-rover-mppi-isaacsim_amd/csrc``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPPI_LIB_PATH: an alternative build of the same library (diagnostic A/B builds)
LIB_PATH = os.environ.get("MPPI_LIB_PATH") or os.path.join(_HERE, "libmppi_hip.so")

MPPI_OK = 0
PROJ = {"2d": 2, "3d": 3, 2: 2, 3: 3}


class MppiParams(C.Structure):
    _fields_ = [
        ("num_trajectories", C.c_int64),
        ("k_offset", C.c_int64),
        ("num_iterations", C.c_int32),
        ("reserved0", C.c_int32),
        ("dt", C.c_float),
        ("robot_radius", C.c_float),
        ("min_u1", C.c_float), ("max_u1", C.c_float),
        ("min_u2", C.c_float), ("max_u2", C.c_float),
        ("v_min_linear", C.c_float), ("v_max_linear", C.c_float),
        ("v_min_angular", C.c_float), ("v_max_angular", C.c_float),
        ("temperature", C.c_float),
        ("filter_k", C.c_float), ("filter_a", C.c_float),
        ("opt_filter_k", C.c_float), ("opt_filter_a", C.c_float),
        ("wheel_offset", C.c_float),
        ("w_path", C.c_float), ("w_slope", C.c_float), ("w_speed", C.c_float),
        ("w_obstacle", C.c_float),
        ("collision_threshold", C.c_float), ("collision_penalty", C.c_float),
        ("horizon", C.c_float),
        ("seed", C.c_uint64),
    ]


class MppiState(C.Structure):
    _fields_ = [
        ("x", C.c_float), ("y", C.c_float),
        ("heading", C.c_float * 3),
        ("left_wheel_speed", C.c_float), ("right_wheel_speed", C.c_float),
        ("goal_x", C.c_float), ("goal_y", C.c_float),
        ("std_dev_u1", C.c_float), ("std_dev_u2", C.c_float),
    ]


_FP = C.POINTER(C.c_float)
_DP = C.POINTER(C.c_double)


class MppiOutputs(C.Structure):
    _fields_ = [(n, _FP) for n in ("u1_opt", "u2_opt", "lin_vel", "ang_vel", "traj_sim",
                                   "heading_sim", "left_wheel_sim", "right_wheel_sim")]


# name -> (restype, argtypes); must match include/mppi.h (tests/test_lib_symbols.py checks both ways)
_PROTOS = {
    "mppi_abi_version": (C.c_int, []),
    "mppi_last_error": (C.c_char_p, []),
    "mppi_create": (C.c_int, [C.POINTER(MppiParams), C.c_int32, C.POINTER(C.c_void_p)]),
    "mppi_destroy": (None, [C.c_void_p]),
    "mppi_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mppi_set_dem": (C.c_int, [C.c_void_p, _FP, C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float]),
    "mppi_dem_updated": (C.c_int, [C.c_void_p]),
    "mppi_set_dem_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_float,
                                      C.c_float, C.c_float]),
    "mppi_set_costmap": (C.c_int, [C.c_void_p, _FP, C.c_int32, C.c_float, C.c_float]),
    "mppi_set_state": (C.c_int, [C.c_void_p, C.POINTER(MppiState)]),
    "mppi_set_nominal": (C.c_int, [C.c_void_p, _FP, _FP]),
    "mppi_get_nominal": (C.c_int, [C.c_void_p, _FP, _FP]),
    "mppi_step": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint64, C.POINTER(MppiOutputs)]),
    "mppi_step_injected": (C.c_int, [C.c_void_p, C.c_int32, _FP, _FP, C.POINTER(MppiOutputs)]),
    "mppi_set_async_tail": (C.c_int, [C.c_void_p, C.c_int32]),
    "mppi_get_outputs": (C.c_int, [C.c_void_p, C.POINTER(MppiOutputs)]),
    "mppi_record_len": (C.c_int64, [C.c_void_p]),
    "mppi_step_partial": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint64, C.c_void_p]),
    "mppi_step_finish": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(MppiOutputs)]),
    "mppi_get_costs": (C.c_int, [C.c_void_p, _FP, C.c_int64]),
    "mppi_dump_rollouts": (C.c_int, [C.c_void_p] + [_FP] * 8),
    "mppi_set_timing": (C.c_int, [C.c_void_p, C.c_int32]),
    "mppi_set_option": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int64]),
    "mppi_get_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                  C.POINTER(C.c_int64)]),
    "mppi_get_tail_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "mppi_get_launch_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int32]),
    "mppi_get_chain_clock": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_int32]),
    "mppi_get_server_time": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                       C.POINTER(C.c_int64)]),
    "mppi_bilinear_query": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]),
    "mppi_selftest": (C.c_int, [C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.POINTER(C.c_int64)]),
    "mppi_bilinear_tiles": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    "mppi_bin_queries": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_void_p]),
    "mppi_bilinear_tiled": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mppi_sync": (C.c_int, [C.c_void_p]),
    "mppi_debug_hold": (C.c_int, [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int32]),
    "mppi_build_costmap": (C.c_int, [C.c_void_p, _DP, C.c_int32, C.c_int32, C.c_double, C.c_double,
                                     C.c_double, C.c_double, C.c_int32, _FP, C.c_int32]),
    "mppi_costmap_builder_create": (C.c_int, [C.c_int32, C.POINTER(C.c_void_p)]),
    "mppi_costmap_builder_destroy": (None, [C.c_void_p]),
    "mppi_costmap_builder_build": (C.c_int, [C.c_void_p, _DP, C.c_int32, C.c_int32, C.c_double, C.c_double,
                                             C.c_double, C.c_double, C.c_int32, _FP, C.c_void_p, C.c_int32]),
    "mppi_costmap_builder_last_ms": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "mppi_group_create": (C.c_int, [C.POINTER(MppiParams), C.c_int32, C.POINTER(C.c_int32),
                                    C.POINTER(C.c_void_p)]),
    "mppi_group_destroy": (None, [C.c_void_p]),
    "mppi_group_size": (C.c_int, [C.c_void_p]),
    "mppi_group_context": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]),
    "mppi_group_shard": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "mppi_group_step": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint64, C.POINTER(MppiOutputs)]),
    "mppi_group_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int32]),
    "mppi_group_selftest": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int64)]),
    "mppi_rollout_python25d": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, _DP, _DP, _DP, _DP, _DP, C.c_double,
                                         C.c_double, C.c_double, C.c_double, _DP, C.POINTER(C.c_int32)]),
}

_lib = None


def load_library(path: str = LIB_PATH):
    """Load libmppi_hip.so and declare its prototypes (raises if it is missing)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"HIP engine library not found at {path}; build it with "
            "`make -C husky-rover-mppi-isaacsim_amd/csrc` (no CPU fallback exists)")
    # PyTorch-ROCm bundles its own libamdhip64.so.7.  Load it first so that the
    # engine's NEEDED libamdhip64.so.7 resolves to the same runtime: a second
    # HIP/HSA runtime in the process would make torch.cuda fail to initialise
    # ("No HIP GPUs are available") once the engine has claimed the device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mppi_abi_version() != 1:
        raise RuntimeError("libmppi_hip.so ABI mismatch")
    if path == LIB_PATH:
        _lib = lib
    return lib


def _fp(a):
    return a.ctypes.data_as(_FP)


def _obstacles(obstacles):
    """Obstacle list [(x_global, y_global, r_obs), ...] -> contiguous float64 [n, 3] (n may be 0)."""
    a = np.ascontiguousarray(np.asarray(obstacles, dtype=np.float64).reshape(-1, 3))
    return a, a.ctypes.data_as(_DP)


COSTMAP_METRICS = {"chamfer": 0, "exact": 1, "chamfer_raster": 2}   # mppi_costmap_metric (include/mppi.h)


def _metric(m):
    if m not in COSTMAP_METRICS:
        raise ValueError(f"costmap metric must be one of {sorted(COSTMAP_METRICS)}, got {m!r}")
    return COSTMAP_METRICS[m]


class CostmapBuilder:
    """Surface.create_obstacles_costmap (MPPI_isaac.py:361-378) on the GPU, no controller context needed.

    build(...) returns the size x size float32 costmap as an ndarray (the reference returns one);
    with out_device=<pointer> the map is written to caller-owned device memory instead.
    """

    def __init__(self, device: int = 0):
        self.lib = load_library()
        self.device = int(device)
        h = C.c_void_p()
        _check(self.lib, self.lib.mppi_costmap_builder_create(self.device, C.byref(h)),
               "mppi_costmap_builder_create")
        self.h = h

    def build(self, obstacles, origin, size, half_width, r_robot, power=20, out_device=None, metric="chamfer"):
        """metric "chamfer": the reference's cv2.distanceTransform(DIST_L2, 5); "exact": exact EDT."""
        obs, optr = _obstacles(obstacles)
        out = None if out_device is not None else np.empty((size, size), np.float32)
        _check(self.lib, self.lib.mppi_costmap_builder_build(
            self.h, optr, obs.shape[0], int(size), float(half_width), float(origin[0]), float(origin[1]),
            float(r_robot), int(power), None if out is None else _fp(out),
            None if out_device is None else C.c_void_p(int(out_device)), _metric(metric)),
            "mppi_costmap_builder_build")
        return out

    def last_ms(self):
        ms = C.c_double()
        _check(self.lib, self.lib.mppi_costmap_builder_last_ms(self.h, C.byref(ms)), "mppi_costmap_builder_last_ms")
        return ms.value

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.lib.mppi_costmap_builder_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _check(lib, rc, what):
    if rc != MPPI_OK:
        msg = lib.mppi_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def make_params(K, H, k_offset=0, **kw):
    """Fill mppi_params; float fields are rounded to float32 by ctypes."""
    p = MppiParams()
    p.num_trajectories = int(K)
    p.k_offset = int(k_offset)
    p.num_iterations = int(H)
    defaults = dict(dt=0.045, robot_radius=1.2, min_u1=-1.0, max_u1=1.0, min_u2=-1.0, max_u2=1.0,
                    v_min_linear=0.0, v_max_linear=2.0, v_min_angular=-1.0, v_max_angular=1.0,
                    temperature=0.3, filter_k=3.5, filter_a=0.96, opt_filter_k=3.0, opt_filter_a=0.92,
                    wheel_offset=0.2, w_path=100.5, w_slope=50.5, w_speed=0.5, w_obstacle=25.0,
                    collision_threshold=0.99, collision_penalty=100000.0, horizon=None, seed=42)
    defaults.update({k: v for k, v in kw.items() if v is not None or k != "horizon"})
    if defaults["horizon"] is None:
        defaults["horizon"] = float(defaults["dt"]) * float(defaults["v_max_linear"]) * int(H)
    for k, v in defaults.items():
        if k == "seed":
            p.seed = int(v) & 0xFFFFFFFFFFFFFFFF
        else:
            setattr(p, k, float(v))
    return p


def make_state(x, y, heading=(1.0, 0.0, 0.0), left_wheel_speed=0.0, right_wheel_speed=0.0,
               goal_x=0.0, goal_y=0.0, std_dev_u1=0.25, std_dev_u2=0.25):
    """Fill mppi_state; the heading is normalised in float64 first (MPPI_isaac.py:493)."""
    s = MppiState()
    s.x, s.y = float(x), float(y)
    h = np.asarray(heading, dtype=np.float64)
    h = (h / np.linalg.norm(h)).astype(np.float32)
    for i in range(3):
        s.heading[i] = float(h[i])
    s.left_wheel_speed = float(left_wheel_speed)
    s.right_wheel_speed = float(right_wheel_speed)
    s.goal_x, s.goal_y = float(goal_x), float(goal_y)
    s.std_dev_u1, s.std_dev_u2 = float(std_dev_u1), float(std_dev_u2)
    return s


class Engine:
    """One device context of the HIP MPPI engine (thin, allocation-free per step)."""

    OUT_NAMES = ("u1_opt", "u2_opt", "lin_vel", "ang_vel", "traj_sim", "heading_sim",
                 "left_wheel_sim", "right_wheel_sim")

    def __init__(self, params: MppiParams, device: int = 0, _ctx=None):
        self.lib = load_library()
        self.params = params
        self.H = int(params.num_iterations)
        self.K = int(params.num_trajectories)
        self.device = int(device)
        self._owned = _ctx is None
        if _ctx is None:
            ctx = C.c_void_p()
            _check(self.lib, self.lib.mppi_create(C.byref(params), self.device, C.byref(ctx)), "mppi_create")
        else:
            ctx = _ctx   # a group member: the group destroys it
        self.ctx = ctx
        H = self.H
        self._buf = {n: np.zeros(3 * H if n.endswith("_sim") else H, np.float32) for n in self.OUT_NAMES}
        self._out = MppiOutputs(*[_fp(self._buf[n]) for n in self.OUT_NAMES])
        self._outref = C.byref(self._out)
        self._step_fn = self.lib.mppi_step   # the per-step call, bound once (it sits on the step's host path)
        self._keep = []
        self.async_tail = False

    # ------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "ctx", None) and self.ctx.value:
            if getattr(self, "_owned", True):
                self.lib.mppi_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, rc, what):
        _check(self.lib, rc, what)

    # ------------------------------------------------------------ scene / state
    def set_stream(self, stream_handle):
        self._c(self.lib.mppi_set_stream(self.ctx, C.c_void_p(stream_handle or None)), "mppi_set_stream")

    def set_dem(self, Z, half_width=None, resolution=None, x_min=None, y_min=None):
        Z = np.ascontiguousarray(Z, dtype=np.float32)
        rows, cols = Z.shape
        if resolution is None:
            resolution = 2.0 * half_width / cols
        if x_min is None:
            x_min = -half_width
        if y_min is None:
            y_min = -half_width
        self._c(self.lib.mppi_set_dem(self.ctx, _fp(Z), rows, cols, x_min, y_min, resolution), "mppi_set_dem")

    def set_dem_device(self, ptr, rows, cols, half_width, resolution=None, keepalive=None):
        if resolution is None:
            resolution = 2.0 * half_width / cols
        self._c(self.lib.mppi_set_dem_device(self.ctx, C.c_void_p(int(ptr)), rows, cols, -half_width,
                                             -half_width, resolution), "mppi_set_dem_device")
        self._keep = [keepalive]

    def dem_updated(self):
        """The bound device DEM was written in place: rebuild the per-cell normal table."""
        self._c(self.lib.mppi_dem_updated(self.ctx), "mppi_dem_updated")

    def set_costmap(self, cm, half_width, resolution=None):
        cm = np.ascontiguousarray(cm, dtype=np.float32)
        size = cm.shape[1]
        if resolution is None:
            resolution = 2.0 * half_width / size
        self._c(self.lib.mppi_set_costmap(self.ctx, _fp(cm), size, half_width, resolution), "mppi_set_costmap")

    def build_costmap(self, obstacles, origin, size, half_width, r_robot, power=20, copy_out=True,
                      metric="chamfer"):
        """Surface.create_obstacles_costmap + costmap_wp.assign in one device pass
        (visual_terrain_stack_full_terrain.py:561-563); returns the map if copy_out."""
        obs, optr = _obstacles(obstacles)
        out = np.empty((size, size), np.float32) if copy_out else None
        self._c(self.lib.mppi_build_costmap(self.ctx, optr, obs.shape[0], int(size), float(half_width),
                                            float(origin[0]), float(origin[1]), float(r_robot), int(power),
                                            None if out is None else _fp(out), _metric(metric)),
                "mppi_build_costmap")
        return out

    def rollout_python25d(self, x0, y0, heading, lin_vel, ang_vel, dt, half_width, resolution, bound=20.0):
        """debug.generate_trajectory_25D (debug.py:312-364) for K trajectories on this context's DEM, float64.

        Returns (traj [K, H, 3], valid [K] bool); valid is False where the reference returns None."""
        v = np.ascontiguousarray(lin_vel, np.float64)
        w = np.ascontiguousarray(ang_vel, np.float64)
        K, H = v.shape
        assert w.shape == (K, H)
        x0 = np.ascontiguousarray(np.broadcast_to(np.asarray(x0, np.float64), (K,)))
        y0 = np.ascontiguousarray(np.broadcast_to(np.asarray(y0, np.float64), (K,)))
        hd = np.ascontiguousarray(np.broadcast_to(np.asarray(heading, np.float64).reshape(-1, 3), (K, 3)))
        traj = np.zeros((K, H, 3), np.float64)
        valid = np.zeros(K, np.int32)
        dp = lambda a: a.ctypes.data_as(_DP)  # noqa: E731
        self._c(self.lib.mppi_rollout_python25d(self.ctx, K, H, dp(x0), dp(y0), dp(hd), dp(v), dp(w), float(dt),
                                                float(half_width), float(resolution), float(bound), dp(traj),
                                                valid.ctypes.data_as(C.POINTER(C.c_int32))),
                "mppi_rollout_python25d")
        return traj, valid.astype(bool)

    def set_state(self, state: MppiState):
        self._c(self.lib.mppi_set_state(self.ctx, C.byref(state)), "mppi_set_state")

    def set_nominal(self, u1, u2):
        u1 = np.ascontiguousarray(u1, dtype=np.float32)
        u2 = np.ascontiguousarray(u2, dtype=np.float32)
        assert u1.size == self.H and u2.size == self.H
        self._c(self.lib.mppi_set_nominal(self.ctx, _fp(u1), _fp(u2)), "mppi_set_nominal")

    def get_nominal(self):
        u1 = np.zeros(self.H, np.float32)
        u2 = np.zeros(self.H, np.float32)
        self._c(self.lib.mppi_get_nominal(self.ctx, _fp(u1), _fp(u2)), "mppi_get_nominal")
        return u1, u2

    def _outputs(self):
        H = self.H
        b = self._buf
        return dict(u1_opt=b["u1_opt"].copy(), u2_opt=b["u2_opt"].copy(), lin_vel=b["lin_vel"].copy(),
                    ang_vel=b["ang_vel"].copy(), traj_sim=b["traj_sim"].reshape(H, 3).copy(),
                    heading_sim=b["heading_sim"].reshape(H, 3).copy(),
                    left_wheel_sim=b["left_wheel_sim"].reshape(H, 3).copy(),
                    right_wheel_sim=b["right_wheel_sim"].reshape(H, 3).copy())

    def step(self, proj="3d", step=0, copy=True):
        rc = self._step_fn(self.ctx, PROJ[proj], int(step), self._outref)
        if rc != MPPI_OK:
            self._c(rc, "mppi_step")
        return self._outputs() if copy else None

    def step_injected(self, u1, u2, proj="3d"):
        u1 = np.ascontiguousarray(u1, dtype=np.float32).reshape(-1)
        u2 = np.ascontiguousarray(u2, dtype=np.float32).reshape(-1)
        assert u1.size == self.K * self.H and u2.size == self.K * self.H
        self._c(self.lib.mppi_step_injected(self.ctx, PROJ[proj], _fp(u1), _fp(u2), C.byref(self._out)),
                "mppi_step_injected")
        return self._outputs()

    def set_async_tail(self, on=True):
        """Deferred optimal rollout: step() returns the controls + row 0 of the *_sim arrays;
        outputs() waits for the rest (bitwise identical)."""
        self._c(self.lib.mppi_set_async_tail(self.ctx, 1 if on else 0), "mppi_set_async_tail")
        self.async_tail = bool(on)

    def outputs(self):
        """All outputs of the last step (waits for a deferred optimal rollout)."""
        self._c(self.lib.mppi_get_outputs(self.ctx, C.byref(self._out)), "mppi_get_outputs")
        return self._outputs()

    def record_len(self):
        return int(self.lib.mppi_record_len(self.ctx))

    def step_partial(self, record_ptr, proj="3d", step=0):
        self._c(self.lib.mppi_step_partial(self.ctx, PROJ[proj], int(step), C.c_void_p(int(record_ptr))),
                "mppi_step_partial")

    def step_finish(self, records_ptr, n, copy=True):
        self._c(self.lib.mppi_step_finish(self.ctx, C.c_void_p(int(records_ptr)), int(n), C.byref(self._out)),
                "mppi_step_finish")
        return self._outputs() if copy else None

    # ------------------------------------------------------------ introspection
    def costs(self):
        c = np.zeros(self.K, np.float32)
        self._c(self.lib.mppi_get_costs(self.ctx, _fp(c), self.K), "mppi_get_costs")
        return c

    def dump(self):
        K, H = self.K, self.H
        arrs = dict(traj=np.zeros((K, H, 3), np.float32), hv=np.zeros((K, H, 3), np.float32),
                    lw=np.zeros((K, H, 3), np.float32), rw=np.zeros((K, H, 3), np.float32),
                    v=np.zeros((K, H), np.float32), w=np.zeros((K, H), np.float32),
                    u1=np.zeros((K, H), np.float32), u2=np.zeros((K, H), np.float32))
        self._c(self.lib.mppi_dump_rollouts(self.ctx, *[_fp(arrs[n]) for n in
                                                        ("traj", "hv", "lw", "rw", "v", "w", "u1", "u2")]),
                "mppi_dump_rollouts")
        return arrs

    def set_option(self, name, value):
        """mppi_set_option (include/mppi.h): per-context tuning / test hooks by name."""
        self._c(self.lib.mppi_set_option(self.ctx, name.encode(), int(value)), "mppi_set_option")

    def set_timing(self, on=True):
        """on: False / True (rollout, finish and tail events) or 2 (rollout and finish only)."""
        mode = on if isinstance(on, int) and not isinstance(on, bool) else (1 if on else 0)
        self._c(self.lib.mppi_set_timing(self.ctx, mode), "mppi_set_timing")

    def timing(self):
        r = C.c_double()
        f = C.c_double()
        n = C.c_int64()
        self._c(self.lib.mppi_get_timing(self.ctx, C.byref(r), C.byref(f), C.byref(n)), "mppi_get_timing")
        return r.value, f.value, n.value

    def tail_timing(self):
        t = C.c_double()
        n = C.c_int64()
        self._c(self.lib.mppi_get_tail_timing(self.ctx, C.byref(t), C.byref(n)), "mppi_get_tail_timing")
        return t.value, n.value

    def launch_info(self):
        info = (C.c_int64 * 18)()
        self._c(self.lib.mppi_get_launch_info(self.ctx, info, 18), "mppi_get_launch_info")
        keys = ("reserved", "block", "blocks", "window_cols", "window_rows", "lds_bytes", "finish_kind",
                "finish_records", "finish_ncol", "finish_groups", "ucache_steps", "resident",
                "server_launches", "server_steps", "server_failed_steps", "server_relaunches",
                "server_fallbacks", "cadence_steps")
        return dict(zip(keys, [int(v) for v in info]))

    def server_time(self):
        """mppi_get_server_time: (rollout us summed, step us summed, steps) on the resident server."""
        r, st, n = C.c_double(0), C.c_double(0), C.c_int64(0)
        self._c(self.lib.mppi_get_server_time(self.ctx, C.byref(r), C.byref(st), C.byref(n)), "mppi_get_server_time")
        return r.value, st.value, n.value

    def chain_clock(self):
        """mppi_get_chain_clock: shader MHz, cycles per chain step, chain us and cycles of the last rollout."""
        v = (C.c_double * 10)()
        self._c(self.lib.mppi_get_chain_clock(self.ctx, v, 10), "mppi_get_chain_clock")
        return dict(zip(("shader_mhz", "cycles_per_step", "chain_us", "chain_cycles", "start_to_chain_us",
                         "chain_to_roles_done_us", "leaf_us", "wg_start_spread_us", "wg_end_spread_us",
                         "wg_span_us"), [float(x) for x in v]))

    def selftest(self, what, n=1 << 24, seed=1):
        bad = C.c_int64()
        self._c(self.lib.mppi_selftest(self.ctx, int(what), int(n), int(seed), C.byref(bad)), "mppi_selftest")
        return bad.value

    def bilinear_tiles(self):
        n = C.c_int32()
        self._c(self.lib.mppi_bilinear_tiles(self.ctx, C.byref(n)), "mppi_bilinear_tiles")
        return n.value

    def bin_queries(self, x_ptr, y_ptr, n, xs_ptr, ys_ptr, perm_ptr, off_ptr):
        self._c(self.lib.mppi_bin_queries(self.ctx, C.c_void_p(int(x_ptr)), C.c_void_p(int(y_ptr)), int(n),
                                          C.c_void_p(int(xs_ptr)), C.c_void_p(int(ys_ptr)),
                                          C.c_void_p(int(perm_ptr)), C.c_void_p(int(off_ptr))), "mppi_bin_queries")

    def bilinear_tiled(self, xs_ptr, ys_ptr, off_ptr, h_ptr):
        """Asynchronous on the engine stream (sync() waits)."""
        self._c(self.lib.mppi_bilinear_tiled(self.ctx, C.c_void_p(int(xs_ptr)), C.c_void_p(int(ys_ptr)),
                                             C.c_void_p(int(off_ptr)), C.c_void_p(int(h_ptr))),
                "mppi_bilinear_tiled")

    def sync(self):
        self._c(self.lib.mppi_sync(self.ctx), "mppi_sync")

    def bilinear_query(self, x_ptr, y_ptr, h_ptr, n):
        self._c(self.lib.mppi_bilinear_query(self.ctx, C.c_void_p(int(x_ptr)), C.c_void_p(int(y_ptr)),
                                             C.c_void_p(int(h_ptr)), int(n)), "mppi_bilinear_query")


def debug_hold(device, stream_handle, groups, lds_bytes, microseconds):
    """mppi_debug_hold (test hook): `groups` workgroups holding lds_bytes of LDS each for `microseconds`
    on the given stream (another stream's kernels occupying CUs when a step is posted)."""
    lib = load_library()
    _check(lib, lib.mppi_debug_hold(int(device), C.c_void_p(stream_handle or None), int(groups), int(lds_bytes),
                                    int(microseconds)), "mppi_debug_hold")


class Group:
    """mppi_group (include/mppi.h): one controller over n GPUs from one process.

    Member i is an Engine over the contiguous shard mppi_group_shard(i) of the K trajectories;
    setters broadcast to every member; step() runs every member's rollout (each member's launches
    enqueued by its own thread), all-gathers the records (RCCL between distinct devices, device
    copies when members share one) and returns the outputs.  When every member's shard is a
    power-of-two number of 256-trajectory leaves the member roots are subtrees of the one-context
    tree and the step is bitwise equal to one context over all K; other splits (e.g. 3 members,
    ragged K) run the same float64 combine with a different pairing.
    """

    def __init__(self, params: MppiParams, devices):
        self.lib = load_library()
        self.params = params
        self.H = int(params.num_iterations)
        self.K = int(params.num_trajectories)
        devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        h = C.c_void_p()
        _check(self.lib, self.lib.mppi_group_create(C.byref(params), len(devices), devs, C.byref(h)),
               "mppi_group_create")
        self.h = h
        self.members = []
        for i, d in enumerate(devices):
            ctx = C.c_void_p()
            _check(self.lib, self.lib.mppi_group_context(h, i, C.byref(ctx)), "mppi_group_context")
            b, n = self.shard(i)
            p = MppiParams.from_buffer_copy(params)
            p.num_trajectories = n if n > 0 else 256
            p.k_offset = int(params.k_offset) + b
            self.members.append(Engine(p, d, _ctx=ctx))

    def shard(self, i):
        b, n = C.c_int64(), C.c_int64()
        _check(self.lib, self.lib.mppi_group_shard(self.h, int(i), C.byref(b), C.byref(n)), "mppi_group_shard")
        return b.value, n.value

    def __len__(self):
        return len(self.members)

    def info(self):
        """mppi_group_info: members, distinct devices, RCCL in use, RCCL ranks, member threads, their spin
        (us) and the granted CPUs."""
        v = (C.c_int64 * 7)()
        _check(self.lib, self.lib.mppi_group_info(self.h, v, 7), "mppi_group_info")
        return dict(zip(("members", "devices", "rccl", "rccl_ranks", "threaded", "spin_us", "granted_cpus"),
                        [int(x) for x in v]))

    def _each(self, name, *a, **kw):
        for m in self.members:
            getattr(m, name)(*a, **kw)

    def set_dem(self, *a, **kw):
        self._each("set_dem", *a, **kw)

    def set_costmap(self, *a, **kw):
        self._each("set_costmap", *a, **kw)

    def set_state(self, state: MppiState):
        self._each("set_state", state)

    def set_nominal(self, u1, u2):
        self._each("set_nominal", u1, u2)

    def set_async_tail(self, on=True):
        """Deferred optimal rollout on every member (Engine.set_async_tail)."""
        self._each("set_async_tail", on)

    def step(self, proj="3d", step=0, copy=True):
        m0 = self.members[0]
        _check(self.lib, self.lib.mppi_group_step(self.h, PROJ[proj], int(step), C.byref(m0._out)),
               "mppi_group_step")
        return m0._outputs() if copy else None

    def outputs(self):
        """All outputs of the last step (every member's deferred optimal rollout waited for)."""
        for m in self.members[1:]:
            m.outputs()
        return self.members[0].outputs()

    def costs(self):
        """Every trajectory's cost in global order (the members' shards concatenated)."""
        return np.concatenate([m.costs()[:self.shard(i)[1]] for i, m in enumerate(self.members)])

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            for m in self.members:
                m.close()
            self.lib.mppi_group_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
