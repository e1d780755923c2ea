"""Mirror of astro_sph_tools.tools (only the projection path is in scope)."""
from . import projections  # noqa: F401
