"""Mirror of astro_sph_tools.tools: the projection path and the periodic-box helpers it
uses (tools/__init__.py:5; _ArrayReorder is outside the hot path)."""
from . import projections  # noqa: F401
from ._periodic_box_manipulations import (calculate_wrapped_displacement,  # noqa: F401
                                          calculate_wrapped_distance, make_periodic,
                                          calculate_periodic, shift_origin, shift_centre)
