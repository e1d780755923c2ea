#!/usr/bin/env python3
"""Generate the golden fixture G8 by RUNNING THE REFERENCE's periodic-box helpers in this
container (tools/_periodic_box_manipulations.py:10-72).

Test infrastructure only; reads /root/reference at run time (container only), writes
``g8_periodic.npz`` next to this file.  The module imports ``unyt`` at its top (not
installed here) and registers unyt overloads with ``functools.singledispatch``; the NumPy
function bodies are extracted with ``ast`` -- the functions named below, their
decorators dropped, the unyt-registered ``_`` overloads left out -- and executed
unmodified with NumPy in scope (the recipe make_golden.py uses for ``_projector.py``).

Inputs (seeded): box width L = 7.3 (not a power of two), coordinates spread over
[-1.3 L, 2.3 L) so that some lie more than one box out (the reference wraps once), plus
the edge values 0, L, L/2, -L/2, their neighbours one ulp away and -0.0.

Usage:  python tests/golden/make_golden_periodic.py
"""
from __future__ import annotations

import ast
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("ASP_REFERENCE", "/root/reference")
SRC = os.path.join(REF, "src/astro_sph_tools/tools/_periodic_box_manipulations.py")
NAMES = ("calculate_wrapped_displacement", "calculate_wrapped_distance", "make_periodic",
         "calculate_periodic", "shift_origin", "shift_centre")


def load_reference():
    tree = ast.parse(open(SRC).read())
    fns = []
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in NAMES:
            node.decorator_list = []
            fns.append(node)
    assert sorted(f.name for f in fns) == sorted(NAMES), [f.name for f in fns]
    ns = {"np": np}
    exec(compile(ast.Module(body=fns, type_ignores=[]), SRC, "exec"), ns)
    return ns


def main():
    ref = load_reference()
    L = 7.3
    rng = np.random.default_rng(8)
    edge = np.array([0.0, -0.0, L, L / 2, -L / 2, np.nextafter(L, 0), np.nextafter(L, 2 * L),
                     np.nextafter(0.0, 1), np.nextafter(0.0, -1), np.nextafter(L / 2, 0),
                     np.nextafter(-L / 2, 0), np.nextafter(-L / 2, -L), 1e-300, -1e-300,
                     2 * L, -L, 3.0 * L - 1e-9])
    pos = rng.uniform(-1.3 * L, 2.3 * L, (1200, 3))
    pos[: edge.size, 0] = edge
    pos[: edge.size, 1] = edge[::-1]
    pos[edge.size: 2 * edge.size, 2] = edge
    centre = np.array([1.3, 6.1, -2.4])
    frm = rng.uniform(-0.5 * L, 1.5 * L, (1200, 3))
    frm[: edge.size, 0] = edge
    to = rng.uniform(-0.5 * L, 1.5 * L, (1200, 3))
    one = rng.uniform(0, L, 3)
    out = dict(L=np.float64(L), pos=pos, centre=centre, frm=frm, to=to, one=one)
    for oic in (False, True):
        k = int(oic)
        out[f"periodic_{k}"] = ref["calculate_periodic"](pos, L, oic)
        mp = pos.copy()
        ref["make_periodic"](mp, L, oic)
        out[f"make_periodic_{k}"] = mp
        out[f"shift_origin_{k}"] = ref["shift_origin"](pos, centre, L, oic)
        out[f"shift_centre_{k}"] = ref["shift_centre"](pos, centre, L, oic)
    out["disp"] = ref["calculate_wrapped_displacement"](frm, to, L)
    out["disp_one"] = ref["calculate_wrapped_displacement"](one, to, L)
    out["dist"] = ref["calculate_wrapped_distance"](frm, to, L)
    out["dist2"] = ref["calculate_wrapped_distance"](frm, to, L, do_squared_distance=True)
    out["dist_one"] = ref["calculate_wrapped_distance"](one, to, L)
    out["dist_vec"] = np.float64(ref["calculate_wrapped_distance"](one, to[0], L))
    np.savez_compressed(os.path.join(HERE, "g8_periodic.npz"), **out)
    print("g8_periodic.npz written:", sorted(out))


if __name__ == "__main__":
    main()
