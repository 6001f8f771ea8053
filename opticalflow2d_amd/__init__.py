"""opticalflow2d_amd — MI355X-native 2-D deformable registration.

A drop-in for the PDE-iteration hot path of tjwdraper/OpticalFlow2d: the
reference's MEX entry point (:func:`OpticalFlow2d`, five call modes) and
``SolverOptions`` enums over a C-ABI (``include/of2d.h``) whose registration
loop runs in hand-written gfx950 HIP kernels (``opticalflow2d_amd/csrc``).
"""
from ._lib import Of2dError, InvalidArgument, build, lib
from .registration import (ImageRegistration, MotionAccumulation, OpticalFlow2d,
                           Regularisation, Verbose, set_print_sink)
from .slab import SlabGroup, SlabSolver, slab_bounds

__all__ = ["OpticalFlow2d", "ImageRegistration", "Regularisation", "Verbose",
           "MotionAccumulation", "set_print_sink", "SlabSolver", "SlabGroup", "slab_bounds", "Of2dError",
           "InvalidArgument", "build", "lib"]
