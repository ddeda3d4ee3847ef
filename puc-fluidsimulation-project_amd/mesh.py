"""Mesh loaders and boundary bookkeeping with the reference's semantics.

readNode / readEle / readPoly keep the reference's names, return dtypes and parsing rules
(StokesColor.py:54-95, poisson.py:27-97): header line, exactly N (or T) records, 1-based ids
converted to 0-based, non-zero boundary markers kept, trailing ``#`` lines ignored.  They read the
whole record block at once (numpy) instead of line by line, so a 14M-node mesh loads in seconds.
"""
from __future__ import annotations

import ctypes as ct
import os
from dataclasses import dataclass, field

import numpy as np
from scipy.spatial import KDTree

from . import _lib

TOL = 1e-6
OUTER_BOUNDARY_MARKER = 1
INNER_BOUNDARY_MARKER = 2
DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def _records(f, n):
    lines = [f.readline() for _ in range(n)]
    return lines


def readNode(filepath, dtype=np.float64):
    """StokesColor.py:54-78 (dtype float64) / poisson.py:27-56 (dtype float32, poisson.py:40).
    Returns (nodes_coords (N,2) dtype, nodes_boundary_markers (N,) int32)."""
    with open(filepath) as f:
        n = int(f.readline().split()[0])
        lines = _records(f, n)
    tok = [l.split() for l in lines]
    if any(len(t) < 4 for t in tok):
        raise ValueError(f"{filepath}: expected {n} records of 'id x y marker'")
    idx = np.array([int(t[0]) for t in tok], dtype=np.int64) - 1
    xy = np.array([[float(t[1]), float(t[2])] for t in tok], dtype=np.float64)
    mk = np.array([int(t[3]) for t in tok], dtype=np.int32)
    coords = np.zeros((n, 2), dtype=dtype)
    markers = np.zeros(n, dtype=np.int32)
    coords[idx] = xy.astype(dtype)  # float64 -> float32 rounds exactly like element assignment
    nz = mk != 0
    markers[idx[nz]] = mk[nz]
    return coords, markers


def readEle(filepath):
    """StokesColor.py:82-95: (T,3) int32, 0-based, rows in file order."""
    with open(filepath) as f:
        t = int(f.readline().split()[0])
        lines = _records(f, t)
    arr = np.array([[int(v) for v in l.split()[1:4]] for l in lines], dtype=np.int64)
    return (arr - 1).astype(np.int32)


def readPoly(path):
    """poisson.py:76-97: skips line 1 (vertex header of a Triangle output .poly), then segments."""
    with open(path) as f:
        f.readline()
        ns = int(f.readline().split()[0])
        seg = np.zeros((ns, 2), dtype=int)
        sm = np.zeros(ns, dtype=int)
        for _ in range(ns):
            p = f.readline().split()
            i = int(p[0]) - 1
            seg[i] = (int(p[1]) - 1, int(p[2]) - 1)
            if len(p) > 3:
                sm[i] = int(p[3])
    return seg, sm


def writeNode(filepath, coords, markers, comment=None):
    """Triangle .node writer (round-trips through readNode bit-exactly: repr of fp64)."""
    with open(filepath, "w") as f:
        f.write(f"{len(coords)}  2  0  1\n")
        for i, ((x, y), m) in enumerate(zip(np.asarray(coords, dtype=np.float64), markers)):
            f.write(f"{i + 1:6d}  {float(x)!r}  {float(y)!r}  {int(m)}\n")
        if comment:
            f.write(f"# {comment}\n")


def writeEle(filepath, triangles, comment=None):
    with open(filepath, "w") as f:
        f.write(f"{len(triangles)}  3  0\n")
        for i, (a, b, c) in enumerate(np.asarray(triangles)):
            f.write(f"{i + 1:6d}  {a + 1:6d}  {b + 1:6d}  {c + 1:6d}\n")
        if comment:
            f.write(f"# {comment}\n")


def writePoly(filepath, segments, segment_markers):
    """Triangle output-style .poly (0 vertices, segments, 0 holes) as readPoly expects."""
    with open(filepath, "w") as f:
        f.write("0  2  0  1\n")
        f.write(f"{len(segments)}  1\n")
        for i, ((a, b), m) in enumerate(zip(segments, segment_markers)):
            f.write(f"{i + 1:6d}  {a + 1:6d}  {b + 1:6d}  {int(m)}\n")
        f.write("0\n")


def find_boundary_pairs(nodes_coords, L=1.0, tol=TOL):
    """StokesColor.py:169-203: each left (x~0) node with the right (x~L) node of nearest y.
    Uses scipy's KDTree one query at a time exactly as the reference does, so exact y-ties
    (mesh2.1 node 260) resolve identically.  Returns an (P,2) int64 array (master, slave)."""
    X = np.asarray(nodes_coords)
    left = np.where(np.abs(X[:, 0]) < tol)[0]
    right = np.where(np.abs(X[:, 0] - L) < tol)[0]
    if len(left) == 0 or len(right) == 0:
        return np.zeros((0, 2), dtype=np.int64)
    tree = KDTree(X[right, 1].reshape(-1, 1))
    # one batched query: each point is searched exactly as a single query would be (same tree, same
    # tie rule), so the pairs are the reference's one-query-per-node loop's
    _, j = tree.query(X[left, 1].reshape(-1, 1))
    return np.stack([left, right[np.asarray(j, dtype=np.int64)]], 1).astype(np.int64)


def filter_wall_pairs(nodes_coords, pairs, tol=TOL, H=1.0):
    """StokesColor.py:449-457: drop pairs whose master lies on y=0 or y=H."""
    if len(pairs) == 0:
        return np.zeros((0, 2), dtype=np.int64)
    y = np.asarray(nodes_coords)[pairs[:, 0], 1]
    keep = ~((np.abs(y - 0.0) < tol) | (np.abs(y - H) < tol))
    return np.ascontiguousarray(pairs[keep], dtype=np.int64)


def boundary_sets(nodes_coords, markers, tol=TOL, H=1.0):
    """StokesColor.py:461-464: (wall, inner, dirichlet, interior) index arrays."""
    X = np.asarray(nodes_coords)
    y = X[:, 1]
    # np.isclose(y, v, atol=tol) on finite values is |y - v| <= atol + rtol |v| (rtol 1e-5), written out:
    # the same test, without isclose's inf / nan bookkeeping over every node (0.3 s at L7)
    wall = np.where((np.abs(y - 0.0) <= tol + 1e-5 * 0.0) | (np.abs(y - H) <= tol + 1e-5 * abs(H)))[0]
    inner = np.where(markers == INNER_BOUNDARY_MARKER)[0]
    mask = np.zeros(X.shape[0], dtype=bool)
    mask[wall] = True
    mask[inner] = True
    dirichlet = np.flatnonzero(mask)  # = np.union1d(wall, inner), sorted
    interior = np.flatnonzero(~mask)
    return wall, inner, dirichlet, interior


@dataclass
class Mesh:
    """A Triangle mesh: coords (N,2), markers (N,), triangles (T,3) 0-based CCW."""

    coords: np.ndarray
    markers: np.ndarray
    triangles: np.ndarray
    name: str = ""
    segments: np.ndarray | None = field(default=None, repr=False)
    segment_markers: np.ndarray | None = field(default=None, repr=False)
    base: "Mesh | None" = field(default=None, repr=False)  # coarse mesh this one was red-refined from
    levels: int = 0                                         # number of red refinements from `base`

    @property
    def N(self):
        return self.coords.shape[0]

    @property
    def T(self):
        return self.triangles.shape[0]

    @classmethod
    def from_files(cls, node_path, ele_path, dtype=np.float64):
        X, mk = readNode(node_path, dtype)
        return cls(X, mk, readEle(ele_path), name=os.path.basename(node_path))

    def as_fp32(self):
        """The mesh as poisson.py / heatEq.py see it (fp32 coordinates, poisson.py:40)."""
        return Mesh(self.coords.astype(np.float32), self.markers, self.triangles, self.name + "/fp32")

    def refined(self, levels):
        """Red refinement (every triangle -> 4, edge midpoints appended; C++ host runtime)."""
        if levels == 0:
            return self
        X = np.ascontiguousarray(self.coords, dtype=np.float64)
        mk = np.ascontiguousarray(self.markers, dtype=np.int32)
        T = np.ascontiguousarray(self.triangles, dtype=np.int32)
        L = _lib.lib()
        n2, t2 = ct.c_int64(), ct.c_int64()
        args = (X.shape[0], _lib.dptr(X), _lib.iptr(mk), T.shape[0], _lib.iptr(T), levels)
        _lib.check(L.pucfem_refine(*args, ct.byref(n2), ct.byref(t2), None, None, None))
        Xo = np.empty((n2.value, 2))
        mko = np.empty(n2.value, dtype=np.int32)
        To = np.empty((t2.value, 3), dtype=np.int32)
        _lib.check(L.pucfem_refine(*args, ct.byref(n2), ct.byref(t2), _lib.dptr(Xo), _lib.iptr(mko), _lib.iptr(To)))
        root = self.base if self.base is not None else self
        return Mesh(Xo, mko, To, name=f"{self.name}+L{levels}", base=root, levels=self.levels + levels)


def load_mesh(name="fine", refine=0):
    """Bundled reference meshes: 'mesh1' (code/mesh/mesh.1 = resources/mesh5.1), 'mesh21'
    (resources/mesh2.1), 'fine' (resources/mesh_fine.1); optionally red-refined `refine` times
    (L5 = 894,208 nodes, L7 = 14,230,528 nodes from 'fine')."""
    d = np.load(os.path.join(DATA, f"{name}.npz"))
    m = Mesh(d["coords"], d["markers"], d["triangles"], name=name, segments=d["segments"],
             segment_markers=d["segment_markers"])
    return m.refined(refine)
