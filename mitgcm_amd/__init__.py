"""mitgcm_amd -- MI355X-native implementation of MITgcm's dynamical hot path.

DYNAMICS (flux-form momentum + TIMESTEP/AB2) and SOLVE_FOR_PRESSURE (CG2D)
as hand-written gfx950 HIP kernels behind a C-ABI (include/mitgcm_amd.h),
with a host driver mirroring the reference's FORWARD_STEP sequence.
"""
from ._lib import MgcmError, lib  # noqa: F401
from .grid import Grid  # noqa: F401
from .model import Model, dynstat  # noqa: F401
from .topology import LatLonTopology  # noqa: F401
