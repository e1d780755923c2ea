#!/usr/bin/env python3
"""Golden G11: the reference's OWN usage example, run by the reference in this container.

Test infrastructure only (reads /root/reference at run time; never travels to the GPU box).
The configuration is the one the reference's author wrote at the end of
src/astro_sph_tools/tools/projections/_projector.py:122-155 -- positions uniform in a
100^3 box, smoothing lengths uniform in [0, 10) (near-zero footprints next to ones 80
pixels wide), a NON-SQUARE (200, 300) image (quirk S2: y corners run to 150 with the
y pitch 100/200, the cull pitch 100/300), chunk 50, Z axis, x, y in [0, 100] -- at a
reduced particle count (2e4 instead of 1e6; the reference's CPU loop is the bottleneck)
and with a seeded generator.  Raw float64 inputs (not float32-rounded), as the demo has.

Recorded, from the reference's create_image / process_chunk / calculate_pixel_value
(built and executed exactly as make_golden.py does):
  img     -- the map with the reference's default kernel (quartic_spline_kernel), A = demo
             properties (uniform [0, 1))
  counts  -- per-pixel neighbour counts: the same call with A = 1 and a kernel_func that
             returns ones (sum of float64 ones: exact integers)

Usage:  python tests/golden/make_golden_demo.py   (~1-2 minutes)
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import build_reference  # noqa: E402

N = 20_000
IMAGE_SIZE = (200, 300)
CHUNK = 50
EXTENT = (0.0, 100.0, 0.0, 100.0)


def demo_inputs(n=N, seed=2024):
    """_projector.py:124-127 with a seeded generator: rand(n, 3) * 100, rand(n) * 10,
    rand(n)."""
    rng = np.random.default_rng(seed)
    positions = rng.random((n, 3)) * 100
    smoothing_lengths = rng.random(n) * 10
    particle_properties = rng.random(n)
    return positions, smoothing_lengths, particle_properties


def ones_kernel(r, h):
    return np.ones_like(np.asarray(r, dtype=np.float64))


def main():
    t0 = time.time()
    ref, Axes, _ = build_reference()
    create_image = ref["create_image"]
    pos, h, A = demo_inputs()
    img = create_image(pos, h, A, IMAGE_SIZE, CHUNK, Axes.Z, *EXTENT)
    t_img = time.time() - t0
    counts = create_image(pos, h, np.ones_like(h), IMAGE_SIZE, CHUNK, Axes.Z, *EXTENT,
                          kernel_func=ones_kernel)
    assert np.array_equal(counts, np.round(counts))
    np.savez_compressed(os.path.join(HERE, "g11_reference_demo.npz"), pos=pos, h=h, A=A,
                        size=np.array(IMAGE_SIZE), cs=CHUNK, axis=2, ext=np.array(EXTENT),
                        img=img, counts=counts.astype(np.int64), seconds=t_img)
    print(f"G11 written in {time.time() - t0:.1f}s: {int(counts.sum())} pairs, "
          f"{int((counts > 0).sum())} covered pixels of {counts.size}")


if __name__ == "__main__":
    main()
