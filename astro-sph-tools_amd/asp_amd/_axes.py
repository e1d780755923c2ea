"""Projection-axis enum, mirroring the reference's ``CoordinateAxes``
(/root/reference/src/astro_sph_tools/_CoordinateAxes.py:3-32): X/Y/Z = 0/1/2,
``str()`` -> "x"/"y"/"z", ``from_string``."""
from enum import Enum


class CoordinateAxes(Enum):
    X = 0
    Y = 1
    Z = 2

    def __str__(self) -> str:
        return "xyz"[self.value]

    @staticmethod
    def from_string(value: str) -> "CoordinateAxes":
        v = value.strip().lower()
        if v in ("x", "y", "z"):
            return CoordinateAxes("xyz".index(v))
        raise ValueError()


# (u, v) columns of the (N, 3) positions array for each projection axis:
# X -> (y, z), Y -> (x, z), Z -> (x, y)   (_projector.py:38-46, .pyx:20-28)
AXIS_COLUMNS = {0: (1, 2), 1: (0, 2), 2: (0, 1)}


def axis_index(projection_axis) -> int:
    """Resolve any axis spelling the reference accepts.

    The reference tests ``projection_axis == CoordinateAxes.X/Y`` for the cull and
    ``str(projection_axis).encode() == b'x'/b'y'`` in the pixel function; anything else
    falls through to Z in both places.  Accept our enum, the reference's enum (any enum
    with X/Y/Z names), ints 0/1/2 and the strings "x"/"y"/"z".
    """
    name = getattr(projection_axis, "name", None)
    if name in ("X", "Y", "Z"):
        return "XYZ".index(name)
    if isinstance(projection_axis, str):
        s = projection_axis.strip().lower()
        return {"x": 0, "y": 1}.get(s, 2)
    if isinstance(projection_axis, bytes):
        return {b"x": 0, b"y": 1}.get(projection_axis, 2)
    try:
        i = int(projection_axis)
    except (TypeError, ValueError):
        return 2
    return i if i in (0, 1) else 2


def reference_axes(projection_axis):
    """(pixel axis, cull axis) exactly as the reference derives them from ANY value.

    The cull (_projector.py:38-46) compares ``projection_axis == CoordinateAxes.X`` / ``.Y``
    -- true only for the enum members -- and otherwise culls on the Z columns; the pixel
    function (_projector.py:63, _pixel_calculations.pyx:20-28) tests
    ``str(projection_axis).encode()`` against ``b'x'`` / ``b'y'``.  Enum members (this
    package's or the reference's own class) give the same axis twice; an int always means
    Z; the str "x" culls on (x, y) but tests distances on (y, z).
    """
    from enum import Enum
    name = getattr(projection_axis, "name", None)
    cull = "XYZ".index(name) if isinstance(projection_axis, Enum) and name in ("X", "Y") else 2
    try:
        tag = str(projection_axis).encode()
    except Exception:  # noqa: BLE001 -- the reference would raise here as well
        raise TypeError(f"projection_axis {projection_axis!r} has no str()") from None
    pixel = {b"x": 0, b"y": 1}.get(tag, 2)
    return pixel, cull
