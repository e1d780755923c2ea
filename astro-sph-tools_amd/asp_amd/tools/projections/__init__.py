"""Mirror of astro_sph_tools.tools.projections (tools/projections/__init__.py:5-6)."""
from ._projector import (create_image, create_weighted_image, create_periodic_image,  # noqa: F401
                         create_images)
from ._cube import create_cube  # noqa: F401
from ._kernels import (quartic_spline_kernel, cubic_spline_kernel, wendland_c2_kernel,  # noqa: F401
                       indicator_kernel)
