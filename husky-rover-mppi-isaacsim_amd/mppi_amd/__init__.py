"""mppi_amd — MI355X-native MPPI rollout-and-cost engine for the Husky rover controller.

Drop-in for thesis_master/warp_implementation/MPPI_isaac.py (Surface, Robot,
MPPI_Controller); the step runs in hand-written HIP kernels (libmppi_hip.so)
behind a ctypes C-ABI (include/mppi.h).
"""
from . import scene  # noqa: F401

__all__ = ["scene"]
