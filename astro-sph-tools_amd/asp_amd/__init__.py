"""asp_amd -- MI355X-native SPH particle-to-grid projector (drop-in for the map-rendering
path of astro_sph_tools: ``tools.projections.create_image`` / ``quartic_spline_kernel``).

    from asp_amd import CoordinateAxes
    from asp_amd.tools.projections import create_image, quartic_spline_kernel

All projection work runs in libasp_hip.so (hand-written HIP for gfx950) behind the C-ABI
in include/asp.h; there is no CPU fallback.
"""
from ._axes import CoordinateAxes  # noqa: F401
from . import tools  # noqa: F401

__version__ = "0.1.0"
