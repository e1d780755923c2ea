#!/usr/bin/env python3
"""Generate golden fixture G10 by RUNNING THE REFERENCE on raw float64 inputs.

Test infrastructure only (container only; reads /root/reference at run time through
make_golden.build_reference(), which compiles the reference's .pyx files in /tmp and runs
its own process_chunk / create_image bodies).  G1-G7 feed float32-representable inputs;
G10 pins the cases those cannot:

* ``plummer_*``: 4000 Plummer particles with positions, h and A as float64 values that are
  NOT float32-representable, 96^2, chunk 16, Z axis: the image, the per-pixel neighbour
  counts (a kernel_func returning ones, A = 1) and an index checksum (A = index % 4093).
* ``edge_*``: 6000 particles placed at distance exactly 2h (in fp64) from pixel corners and
  moved by -3 .. 3 fp64 ulps, plus particles whose r^2 lies within 1e-10 relative of
  (2h)^2 -- pairs whose float32 rounding alone would flip the reference's decision.
  Counts and index checksum, 64^2, chunk 8.
* ``axes_*``: the reference's axis handling for every spelling a caller can pass: the
  enum members, the str "x" / "y" (the cull reads the Z columns, the pixel test the X / Y
  ones: _projector.py:38-46 vs _pixel_calculations.pyx:20-28), ints (Z) and bytes;
  non-square 40 x 56 image, chunk 12.

Usage:  python tests/golden/make_golden_f64.py   (~1 minute)
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import build_reference, plummer  # noqa: E402


def ones_kernel(r, h):
    """kernel_func for neighbour counting: W = 1 for every pair in the mask."""
    return np.ones(np.asarray(r).shape[0], dtype=np.float64)


def not_f32(a, rng):
    """Perturb float64 values off the float32 grid (a few 1e-9 relative)."""
    a = np.asarray(a, np.float64)
    b = a * (1.0 + rng.uniform(-3e-9, 3e-9, a.shape))
    assert not np.any(b.astype(np.float32).astype(np.float64) == b), "still f32-representable"
    return b


def main():
    t0 = time.time()
    ref, Axes, qsk = build_reference()
    create_image = ref["create_image"]
    out = {}
    rng = np.random.default_rng(101)

    # ---- plummer: raw fp64 -------------------------------------------------------
    n, G, cs, ext = 4000, 96, 16, (-2.0, 2.0, -2.0, 2.0)
    p = plummer(n, seed=17, h_law="knn32")
    pos = not_f32(p["pos"], rng)
    h = not_f32(p["h"], rng)
    A = not_f32(p["m"] * 1e4, rng)
    out.update(plummer_pos=pos, plummer_h=h, plummer_A=A, plummer_size=np.array([G, G]),
               plummer_cs=cs, plummer_ext=np.array(ext))
    out["plummer_img"] = create_image(pos, h, A, (G, G), cs, Axes.Z, *ext)
    out["plummer_cnt"] = create_image(pos, h, np.ones(n), (G, G), cs, Axes.Z, *ext,
                                      kernel_func=ones_kernel)
    ids = (np.arange(n) % 4093).astype(np.float64)
    out["plummer_ids"] = create_image(pos, h, ids, (G, G), cs, Axes.Z, *ext,
                                      kernel_func=ones_kernel)

    # ---- edge: pairs at the 2h boundary in fp64 -----------------------------------
    G2, cs2, ext2 = 64, 8, (-1.0, 1.0, -1.0, 1.0)
    ps = 2.0 / G2
    m = 6000
    xi = rng.integers(4, G2 - 4, m)
    yi = rng.integers(4, G2 - 4, m)
    hh = ps * rng.choice([0.5, 0.75, 1.0, 1.25, 1.5], m) * (1.0 + rng.uniform(-1e-7, 1e-7, m))
    X = -1.0 + xi * ps          # the reference's corner expressions (.pyx:13-14)
    Y = -1.0 + yi * (2.0 / G2)
    ang = rng.uniform(0, 2 * np.pi, m)
    u = X + 2.0 * hh * np.cos(ang)
    v = Y + 2.0 * hh * np.sin(ang)
    k = rng.integers(-3, 4, m)
    u = u + k * np.spacing(u)            # a few fp64 ulps either side
    close = rng.random(m) < 0.4          # r^2 within 1e-10 relative of (2h)^2
    scale = 1.0 + rng.uniform(-1e-10, 1e-10, m)
    u = np.where(close, X + (u - X) * scale, u)
    v = np.where(close, Y + (v - Y) * scale, v)
    pos2 = np.stack([u, v, rng.uniform(-1, 1, m)], 1)
    dx, dy = u - X, v - Y
    r2 = dx * dx + dy * dy
    t = 2.0 * hh
    f32_flip = ((dx.astype(np.float32).astype(np.float64) ** 2 +
                 dy.astype(np.float32).astype(np.float64) ** 2) < (t.astype(np.float32).astype(np.float64)) ** 2) != (r2 < t * t)
    out.update(edge_pos=pos2, edge_h=hh, edge_size=np.array([G2, G2]), edge_cs=cs2,
               edge_ext=np.array(ext2), edge_f32_flips=int(f32_flip.sum()))
    out["edge_cnt"] = create_image(pos2, hh, np.ones(m), (G2, G2), cs2, Axes.Z, *ext2,
                                   kernel_func=ones_kernel)
    ids2 = (np.arange(m) % 4093).astype(np.float64)
    out["edge_ids"] = create_image(pos2, hh, ids2, (G2, G2), cs2, Axes.Z, *ext2,
                                   kernel_func=ones_kernel)

    # ---- axes: every spelling, non-square --------------------------------------
    n3, size3, cs3, ext3 = 1500, (40, 56), 12, (-1.5, 1.5, -1.0, 2.0)
    p3 = plummer(n3, seed=23, h_law="knn32")
    pos3 = not_f32(p3["pos"], rng)
    h3 = not_f32(p3["h"], rng) * 1.5
    A3 = not_f32(p3["T"] / 1e4, rng)
    out.update(axes_pos=pos3, axes_h=h3, axes_A=A3, axes_size=np.array(size3), axes_cs=cs3,
               axes_ext=np.array(ext3))
    spellings = {"enumX": Axes.X, "enumY": Axes.Y, "enumZ": Axes.Z, "strx": "x", "stry": "y",
                 "strz": "z", "strX": "X", "int0": 0, "int1": 1, "bytesx": b"x"}
    for key, ax in spellings.items():
        out[f"axes_img_{key}"] = create_image(pos3, h3, A3, size3, cs3, ax, *ext3)
        out[f"axes_cnt_{key}"] = create_image(pos3, h3, np.ones(n3), size3, cs3, ax, *ext3,
                                              kernel_func=ones_kernel)
    out["axes_keys"] = np.array(list(spellings))

    np.savez_compressed(os.path.join(HERE, "g10_fp64_axes.npz"), **out)
    print(f"G10 written in {time.time() - t0:.1f}s; {out['edge_f32_flips']} edge pairs whose "
          f"float32 rounding flips the decision")


if __name__ == "__main__":
    main()
