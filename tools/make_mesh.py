#!/usr/bin/env python3
"""Write a bundled reference mesh, red-refined L times, as Triangle files (.node/.ele/.poly).

SURVEY.md §8 f2: the synthetic benchmark meshes (L5 = mesh_fine x5, 894,208 nodes; L7 = x7,
14,230,528 nodes) as reproducible artefacts in the reference's own file format, readable by the
reference's readNode / readEle / readPoly (StokesColor.py:54-95, poisson.py:76-97) and by ours.

  python tools/make_mesh.py --mesh fine --level 5 --out /tmp/meshes   -> mesh_fine_L5.{node,ele,poly}

Coordinates are written with repr() of the fp64 values, so readNode returns the refined mesh's
coordinates bit for bit.  Boundary segments are refined with the mesh: each segment (a, b) of the
coarse boundary becomes (a, m), (m, b), m the edge midpoint node the refinement created.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _pkg():
    from importlib import import_module

    return import_module("puc-fluidsimulation-project_amd")


def refine_segments(coarse_coords, segments, markers, fine_coords, levels):
    """Split every boundary segment at the midpoint nodes the red refinement appended, `levels`
    times.  The midpoint of (a, b) is (x_a + x_b) * 0.5 in fp64 (the refiner's arithmetic), so it
    is found by exact coordinate lookup."""
    index = {(float(x), float(y)): i for i, (x, y) in enumerate(np.asarray(fine_coords))}
    X = np.asarray(fine_coords)
    seg = [tuple(map(int, s)) for s in segments]
    mk = [int(m) for m in markers]
    for _ in range(levels):
        nseg, nmk = [], []
        for (a, b), m in zip(seg, mk):
            mid = ((X[a, 0] + X[b, 0]) * 0.5, (X[a, 1] + X[b, 1]) * 0.5)
            c = index.get((float(mid[0]), float(mid[1])))
            if c is None:
                raise ValueError(f"no refinement midpoint for boundary segment ({a}, {b})")
            nseg += [(a, c), (c, b)]
            nmk += [m, m]
        seg, mk = nseg, nmk
    return np.array(seg, dtype=np.int64).reshape(-1, 2), np.array(mk, dtype=np.int64)


def write_mesh(name, level, out_dir):
    """Write `name` refined `level` times to out_dir; returns the three paths."""
    pf = _pkg()
    base = pf.load_mesh(name)
    mesh = pf.load_mesh(name, refine=level)
    seg, segm = refine_segments(base.coords, base.segments, base.segment_markers, mesh.coords, level)
    os.makedirs(out_dir, exist_ok=True)
    stem = os.path.join(out_dir, f"mesh_{name}_L{level}")
    note = f"{name} red-refined {level}x by pucfem ({mesh.N} nodes, {mesh.T} triangles)"
    pf.writeNode(stem + ".node", mesh.coords, mesh.markers, comment=note)
    pf.writeEle(stem + ".ele", mesh.triangles, comment=note)
    pf.writePoly(stem + ".poly", seg, segm)
    return stem + ".node", stem + ".ele", stem + ".poly"


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--mesh", default="fine", choices=["mesh1", "mesh21", "fine"])
    ap.add_argument("--level", type=int, default=5)
    ap.add_argument("--out", default="meshes")
    a = ap.parse_args()
    for p in write_mesh(a.mesh, a.level, a.out):
        print(p, os.path.getsize(p), "bytes")


if __name__ == "__main__":
    main()
