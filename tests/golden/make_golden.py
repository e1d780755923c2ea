#!/usr/bin/env python3
"""Generate the golden fixtures G1-G7 by RUNNING THE REFERENCE in this container.

Test infrastructure only.  Reads /root/reference at run time (container only -- the
reference never travels to the GPU box); writes small ``.npz`` fixtures next to this
file.  Nothing from /root/reference is copied into the repository: the .pyx sources
are copied into a scratch build directory under /tmp and compiled there.

What runs:

* ``_kernels.pyx`` (``quartic_spline_kernel``) -- compiled VERBATIM with Cython.
* ``_pixel_calculations.pyx`` (``calculate_pixel_value``) -- as shipped it does not
  compile under Cython 3.2.9 (crash at :31:41, typed memoryview arithmetic).  The
  survey's typing-only patch is applied: untype the memoryview parameters/locals and
  ``char`` -> ``bytes`` for the axis.  Every arithmetic line (:11-14, :20-34) is
  byte-identical to the reference.
* ``_projector.py`` -- the function bodies of ``process_chunk`` (:13-73) and
  ``create_image`` (:75-120) are extracted from the reference file with ``ast`` and
  executed unmodified.  Their only external name besides numpy is
  ``QuasarCode.Console.print_debug`` (a debug print; QuasarCode is not installed), which
  is bound to a no-op.  ``calculate_pixel_value`` / ``quartic_spline_kernel`` /
  ``CoordinateAxes`` are bound to the compiled reference modules above and the
  reference's own ``_CoordinateAxes.py``.

Recording without modifying the reference: inputs are given pairwise-distinct
smoothing lengths, so the ``h`` arrays the reference hands to ``kernel_func`` (the
neighbour set of a pixel, ``_pixel_calculations.pyx:31-33``) and to
``calculate_pixel_value`` (the culled tile set, ``_projector.py:49-51``) identify the
particles exactly.  The recorders pass every call straight through, so the recorded
images are the reference's own.

All particle inputs are float32-representable float64 so that the GPU path (which is
fed float32 SoA) sees *identical* inputs.

Usage:  python tests/golden/make_golden.py   (takes ~1 minute)
"""
from __future__ import annotations

import ast
import importlib.util
import os
import shutil
import subprocess
import sys
import textwrap
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))
from asp_amd.plummer import plummer  # noqa: E402

REF = os.environ.get("ASP_REFERENCE", "/root/reference")
PROJ = os.path.join(REF, "src/astro_sph_tools/tools/projections")
BUILD = os.environ.get("ASP_GOLDEN_BUILD", "/tmp/asp_golden_build")

# The survey's typing-only patch (Appendix A), as exact single-occurrence replacements.
PYX_PATCH = [
    ("double[:, :] positions, double[:] smoothing_lengths, double[:] particle_properties",
     "object positions, object smoothing_lengths, object particle_properties"),
    ("    cdef double[:] dx, dy\n", "    pass\n"),
    ("    cdef double[:] r2, r, weights\n", "    pass\n"),
    ("    cdef double result = 0.0\n", "    result = 0.0\n"),
    ("char projection_axis,", "bytes projection_axis,"),
]

SETUP_PY = textwrap.dedent("""
    import numpy
    from setuptools import setup, Extension
    from Cython.Build import cythonize
    exts = [Extension(n, [n + ".pyx"], include_dirs=[numpy.get_include()])
            for n in ("_kernels", "_pixel_calculations")]
    # directives = pyproject.toml:76
    setup(ext_modules=cythonize(exts, compiler_directives=dict(
        boundscheck=False, nonecheck=False, language_level=3, binding=True)))
""")


def build_reference():
    os.makedirs(BUILD, exist_ok=True)
    shutil.copyfile(os.path.join(PROJ, "_kernels.pyx"), os.path.join(BUILD, "_kernels.pyx"))
    src = open(os.path.join(PROJ, "_pixel_calculations.pyx")).read()
    for a, b in PYX_PATCH:
        assert src.count(a) == 1, f"patch anchor not unique/found: {a!r}"
        src = src.replace(a, b)
    open(os.path.join(BUILD, "_pixel_calculations.pyx"), "w").write(src)
    open(os.path.join(BUILD, "setup.py"), "w").write(SETUP_PY)
    subprocess.run([sys.executable, "setup.py", "build_ext", "--inplace", "-q"], cwd=BUILD,
                   check=True, stdout=subprocess.DEVNULL)
    sys.path.insert(0, BUILD)
    import _kernels  # noqa: F401
    import _pixel_calculations  # noqa: F401

    spec = importlib.util.spec_from_file_location(
        "_ref_coordinate_axes", os.path.join(REF, "src/astro_sph_tools/_CoordinateAxes.py"))
    axes = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(axes)

    class _NoOpConsole:  # QuasarCode.Console stand-in for debug prints only
        @staticmethod
        def print_debug(*a, **k):
            pass

    tree = ast.parse(open(os.path.join(PROJ, "_projector.py")).read())
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef)
           and n.name in ("process_chunk", "create_image")]
    assert len(fns) == 2
    ns = {"np": np, "Callable": __import__("typing").Callable, "Console": _NoOpConsole,
          "CoordinateAxes": axes.CoordinateAxes,
          "quartic_spline_kernel": _kernels.quartic_spline_kernel,
          "calculate_pixel_value": _pixel_calculations.calculate_pixel_value}
    exec(compile(ast.Module(body=fns, type_ignores=[]), os.path.join(PROJ, "_projector.py"),
                 "exec"), ns)
    return ns, axes.CoordinateAxes, _kernels.quartic_spline_kernel


def f32r(a):
    """Round to the nearest float32 and return float64 (inputs identical for the GPU)."""
    return np.asarray(a, dtype=np.float32).astype(np.float64)


def wendland_c2_numpy(r, h):
    """Build-defined Wendland-C2, support 2h, 3-D normalisation.

    W = 21/(16 pi h^3) (1 - q/2)^4 (1 + 2q), q = r/h < 2.  A plain NumPy callable
    handed to the reference through its ``kernel_func`` plugin point (G6).
    """
    r = np.asarray(r, dtype=np.float64)
    h = np.asarray(h, dtype=np.float64)
    q = r / h
    t = np.clip(1.0 - 0.5 * q, 0.0, None)
    return np.where(q < 2.0, 21.0 / (16.0 * np.pi * h ** 3) * t ** 4 * (1.0 + 2.0 * q), 0.0)


def distinct_h(h, rng):
    """Make smoothing lengths pairwise distinct float32 values (recording key)."""
    h = f32r(h)
    for _ in range(8):
        _, inv, cnt = np.unique(h, return_inverse=True, return_counts=True)
        dup = cnt[inv] > 1
        if not dup.any():
            return h
        h[dup] = f32r(h[dup] * (1.0 + 1e-6 * rng.uniform(0.5, 1.0, dup.sum())))
    raise RuntimeError("could not make h distinct")


def main():
    t0 = time.time()
    ref, Axes, qsk = build_reference()
    create_image = ref["create_image"]
    out = {}

    # ---------------- G1: kernel table (quartic_spline_kernel, verbatim) -------------
    one = np.float64(1.0)
    qs = np.array([0.0, 0.5, np.nextafter(one, 0), 1.0, np.nextafter(one, 2), 1.5,
                   np.nextafter(2.0, 0), 2.0, 3.0])
    hs = np.array([0.5, 1.0, 2.7])
    qq, hh = np.meshgrid(qs, hs, indexing="ij")
    r_tab = (qq * hh).ravel()
    h_tab = hh.ravel().copy()
    rng = np.random.default_rng(1)
    r_rnd = rng.uniform(0.0, 5.0, 10000)
    h_rnd = rng.uniform(0.05, 3.0, 10000)
    r1 = np.concatenate([r_tab, r_rnd])
    h1 = np.concatenate([h_tab, h_rnd])
    np.savez_compressed(os.path.join(HERE, "g1_kernel_table.npz"), r=r1, h=h1, w=qsk(r1, h1))

    # ---------------- G2: hand cases ----------------------------------------------
    cases = []

    def run(pos, h, A, size, cs, axis, ext):
        img = create_image(np.ascontiguousarray(pos, dtype=np.float64), np.asarray(h, np.float64),
                           np.asarray(A, np.float64), size, cs, axis, *ext)
        cases.append(dict(pos=np.asarray(pos, np.float64), h=np.asarray(h, np.float64),
                          A=np.asarray(A, np.float64), size=np.array(size), cs=cs,
                          axis=axis.value, ext=np.array(ext, np.float64), img=img))
        return img

    ext1 = (-1.0, 1.0, -1.0, 1.0)
    img = run([[0.0, 0.0, 0.0]], [0.5], [1.0], (4, 4), 4, Axes.Z, ext1)
    assert abs(img[2, 2] - 2.546479089470) < 1e-9, img[2, 2]
    run([[0.0, 0.0, 0.0]], [0.25], [1.0], (4, 4), 4, Axes.Z, ext1)  # r = 2h = 0.5 at neighbours
    run([[0.5, -0.5, 0.0]], [0.2], [1.0], (4, 4), 2, Axes.Z, ext1)
    run([[0.0, -0.5, 0.0]], [0.2], [1.0], (4, 4), 2, Axes.X, ext1)
    run([[0.5, 0.0, -0.5]], [0.2], [1.0], (4, 4), 3, Axes.Y, ext1)
    run([[0.0, 0.0, 0.0]], [0.3], [2.0], (4, 8), 4, Axes.Z, ext1)   # non-square quirk S2
    run([[0.0, 0.0, 0.0]], [0.3], [2.0], (4, 8), 3, Axes.Z, ext1)   # ... chunk-dependent cull
    run([[0.0, 0.0, 0.0]], [0.3], [2.0], (8, 4), 3, Axes.Z, ext1)
    run([[0.0, 0.0, 0.0]], [0.0], [1.0], (4, 4), 4, Axes.Z, ext1)   # h = 0 -> all zero
    run([[0.1, 0.2, 0.3], [-0.3, 0.1, 0.0], [0.7, 0.7, 0.7]], [0.4, 0.3, 0.25], [1.0, -2.0, 0.5],
        (5, 7), 2, Axes.Z, (-1.0, 1.5, -0.5, 1.0))
    run(np.zeros((0, 3)), np.zeros(0), np.zeros(0), (3, 3), 2, Axes.Z, ext1)  # empty
    g2 = {}
    for i, c in enumerate(cases):
        for k, v in c.items():
            g2[f"c{i}_{k}"] = np.asarray(v)
    g2["n_cases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, "g2_hand_cases.npz"), **g2)

    # ---------------- G3/G4/G5: Plummer 1e4 -> 256^2, Z axis, +-2, chunk 16 ---------
    N, G, CS = 10_000, 256, 16
    p = plummer(N, seed=0, h_law="knn32")
    pos = f32r(p["pos"])
    rng = np.random.default_rng(7)
    h = distinct_h(p["h"], rng)
    A = f32r(p["m"] * 1e4)           # masses of order 1 (A = m)
    ext = (-2.0, 2.0, -2.0, 2.0)
    h_to_idx = {float(v): i for i, v in enumerate(h)}
    assert len(h_to_idx) == N

    # recorders (pass-through): tile membership and sampled-pixel neighbour sets
    n_chunks_side = G // CS
    member = {}
    nbr = {}
    sample_rng = np.random.default_rng(11)
    sample = sample_rng.choice(G * G, size=256, replace=False)
    # bias half of the samples to the dense centre, where neighbour sets are large
    centre = (G // 2 - 20 + sample_rng.integers(0, 40, 128)) * G + (G // 2 - 20 + sample_rng.integers(0, 40, 128))
    sample = np.unique(np.concatenate([sample[:128], centre]))
    sample_set = set(int(s) for s in sample)
    state = {"pix": None}
    real_cpv = ref["calculate_pixel_value"]

    def rec_cpv(xi, yi, P, H, Aa, ax, x0, x1, y0, y1, nx, kf):
        key = (int(xi) // CS, int(yi) // CS)
        if key not in member:
            member[key] = np.sort(np.array([h_to_idx[float(v)] for v in H], dtype=np.int64))
        state["pix"] = int(xi) * G + int(yi)
        return real_cpv(xi, yi, P, H, Aa, ax, x0, x1, y0, y1, nx, kf)

    def rec_kernel(r, hm):
        pix = state["pix"]
        if pix in sample_set:
            nbr[pix] = np.sort(np.array([h_to_idx[float(v)] for v in np.asarray(hm)], dtype=np.int64))
        return qsk(r, hm)

    ref["calculate_pixel_value"] = rec_cpv
    t1 = time.time()
    img3 = create_image(pos, h, A, (G, G), CS, Axes.Z, *ext, kernel_func=rec_kernel)
    t_g3 = time.time() - t1
    ref["calculate_pixel_value"] = real_cpv
    # the recorder must not change the image: compare with a plain run
    img3_plain = create_image(pos, h, A, (G, G), CS, Axes.Z, *ext)
    assert np.array_equal(img3, img3_plain)
    np.savez_compressed(os.path.join(HERE, "g3_plummer_1e4_256.npz"),
                        pos=pos.astype(np.float32), h=h.astype(np.float32), A=A.astype(np.float32),
                        size=np.array([G, G]), cs=CS, axis=2, ext=np.array(ext), img=img3,
                        seconds=t_g3)
    # G4: CSR of culled particle indices per chunk, chunks in (cx, cy) row-major order
    offs, idx = [0], []
    for cx in range(n_chunks_side):
        for cy in range(n_chunks_side):
            m = member.get((cx, cy), np.zeros(0, np.int64))
            idx.append(m)
            offs.append(offs[-1] + len(m))
    np.savez_compressed(os.path.join(HERE, "g4_tile_membership.npz"),
                        offsets=np.array(offs, np.int64), index=np.concatenate(idx).astype(np.int32),
                        chunk_size=CS, n_chunks=np.array([n_chunks_side, n_chunks_side]))
    # G5: neighbour CSR for sampled pixels (pixel id = xi*G + yi)
    pix = np.array(sorted(sample_set), np.int64)
    offs, idx = [0], []
    for q in pix:
        s = nbr.get(int(q), np.zeros(0, np.int64))
        idx.append(s)
        offs.append(offs[-1] + len(s))
    np.savez_compressed(os.path.join(HERE, "g5_neighbours.npz"), pixels=pix,
                        offsets=np.array(offs, np.int64), index=np.concatenate(idx).astype(np.int32))

    # ---------------- G6: Wendland-C2 through kernel_func on G3 inputs -------------
    img6 = create_image(pos, h, A, (G, G), CS, Axes.Z, *ext, kernel_func=wendland_c2_numpy)
    np.savez_compressed(os.path.join(HERE, "g6_wendland_c2.npz"), img=img6)

    # ---------------- G7: X / Y axes, 64^2, and a permuted-input run ---------------
    n7 = 2000
    p7 = plummer(n7, seed=3, h_law="knn32")
    pos7, h7, A7 = f32r(p7["pos"]), f32r(p7["h"]), f32r(p7["T"] / 1e4)
    ext7 = (-1.5, 1.5, -1.5, 1.5)
    g7 = dict(pos=pos7.astype(np.float32), h=h7.astype(np.float32), A=A7.astype(np.float32),
              ext=np.array(ext7), size=np.array([64, 64]), cs=8)
    for ax in (Axes.X, Axes.Y, Axes.Z):
        g7[f"img_{ax.value}"] = create_image(pos7, h7, A7, (64, 64), 8, ax, *ext7)
    perm = np.random.default_rng(5).permutation(n7)
    g7["perm"] = perm
    g7["img_z_perm"] = create_image(pos7[perm], h7[perm], A7[perm], (64, 64), 8, Axes.Z, *ext7)
    # non-square, chunk-dependent (S2 quirk) on real data
    g7["img_ns_48x64_c16"] = create_image(pos7, h7, A7, (48, 64), 16, Axes.Z, *ext7)
    g7["img_ns_64x40_c7"] = create_image(pos7, h7, A7, (64, 40), 7, Axes.Z, *ext7)
    np.savez_compressed(os.path.join(HERE, "g7_axes_permuted.npz"), **g7)

    print(f"golden fixtures written in {time.time() - t0:.1f}s (G3 reference run {t_g3:.2f}s)")


if __name__ == "__main__":
    main()
