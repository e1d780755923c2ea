#!/usr/bin/env python3
"""Generate the golden fixture G9 by RUNNING THE REFERENCE's ionisation-table class in this
container (data_structures/_IonisationTable.py:30-69, ``IonisationTableBase``).

Test infrastructure only; reads /root/reference at run time (container only), writes
``g9_ion_table.npz`` next to this file.  The module's imports pull in the package's
typing scaffolding; the class body is extracted with ``ast`` (its generic base
``IIonisationTable[P]`` dropped, annotations kept as strings) and executed unmodified with
NumPy and scipy's ``RegularGridInterpolator`` in scope -- the recipe make_golden.py uses
for ``_projector.py``.  scipy is the reference's own dependency (pyproject.toml) and is
1.15.3 here.

Inputs (seeded): an HM01-shaped 3-D table over (log10 n_H, log10 T, redshift) with
non-uniform, strictly ascending axes (7 x 9 x 5), log10 ion fractions with a block of
exact zeros; query points spread inside the table, on grid nodes and cell faces, exactly
on the first/last node of each axis, one ulp outside, far outside, and NaN in each
column.  Both ``__call__`` (3 columns) and ``evaluate_at_redshift`` (2 columns + z) are
recorded, the latter at an interior redshift, a node redshift and an out-of-range one.

Usage:  python tests/golden/make_golden_table.py
"""
from __future__ import annotations

import ast
import os

import numpy as np
from scipy.interpolate import RegularGridInterpolator

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("ASP_REFERENCE", "/root/reference")
SRC = os.path.join(REF, "src/astro_sph_tools/data_structures/_IonisationTable.py")


def reference_class():
    tree = ast.parse(open(SRC).read())
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == "IonisationTableBase":
            node.bases = []
            node.keywords = []
            mod = ast.Module(body=[ast.ImportFrom(module="__future__",
                                                  names=[ast.alias(name="annotations")],
                                                  level=0), node], type_ignores=[])
            ns = {"np": np, "RegularGridInterpolator": RegularGridInterpolator}
            exec(compile(ast.fix_missing_locations(mod), SRC, "exec"), ns)
            return ns["IonisationTableBase"]
    raise RuntimeError("IonisationTableBase not found")


def axis(rng, lo, hi, n):
    g = np.sort(rng.uniform(lo, hi, n - 2))
    g = np.concatenate([[lo], g, [hi]])
    assert np.all(np.diff(g) > 0)
    return g


def points(rng, g, n):
    cols = []
    for ax in g:
        lo, hi = ax[0], ax[-1]
        span = hi - lo
        c = rng.uniform(lo, hi, n)
        k = n // 8
        c[:k] = rng.choice(ax, k)                               # on nodes
        c[k:2 * k] = rng.choice([lo, hi], k)                    # on the end nodes
        c[2 * k:2 * k + 4] = [np.nextafter(lo, -np.inf), np.nextafter(hi, np.inf),
                              lo - 0.5 * span, hi + 3 * span]   # just / far outside
        c[2 * k + 4] = np.nan
        cols.append(c)
    P = np.stack(cols, axis=1)
    # shuffle each column independently so edge cases combine across axes
    for d in range(P.shape[1]):
        P[:, d] = P[rng.permutation(n), d]
    return P


def main():
    rng = np.random.default_rng(20261016)
    g = [axis(rng, -8.0, 0.5, 7), axis(rng, 2.0, 8.5, 9), axis(rng, 0.0, 9.0, 5)]
    table = rng.uniform(-12.0, 0.0, (7, 9, 5))
    table[2:4, 3:5, :] = 0.0
    Cls = reference_class()
    ref = Cls(table, *g, redshift_input_index=2)
    P3 = points(rng, g, 512)
    out3 = ref(P3)
    P2 = points(rng, g[:2], 256)
    zs = np.array([3.37, g[2][2], 9.5])
    out2 = np.stack([ref.evaluate_at_redshift(P2, z) for z in zs])
    assert np.isneginf(out3).any() and np.isnan(out3).any()
    np.savez_compressed(os.path.join(HERE, "g9_ion_table.npz"), table=table, g0=g[0], g1=g[1],
                        g2=g[2], points3=P3, out3=out3, points2=P2, redshifts=zs, out2=out2)
    print("wrote g9_ion_table.npz", out3.shape, out2.shape)


if __name__ == "__main__":
    main()
