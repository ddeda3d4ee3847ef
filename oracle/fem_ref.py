"""CPU restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

All citations are into /root/reference (TobiasHoffmannP/PUC-Fluidsimulation-Project @ 2025-09-05).
Per-element loops of the reference are restated with ``np.add.at`` over the
element list in reference order, so the scatter-accumulation order -- and hence
the rounding -- is the reference's.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla
from scipy.spatial import KDTree

__all__ = [
    "read_node", "read_ele", "read_poly", "find_boundary_pairs", "filter_wall_pairs",
    "stiffness", "lumped_mass", "div_area_sum", "divergence", "gradient",
    "fem_system_fp32", "apply_periodic_rowmerge", "apply_dirichlet_rows",
    "boundary_sets", "squirmer_bc", "make_dir_bcu", "make_per_bcu",
    "visc_matrix", "PressureSolver", "centroids", "sl_advect", "mixing_index",
    "plane_coefficients", "locate_bary", "tracer_init", "tracer_step",
    "poisson_literal", "HeatLiteral", "StokesRef", "pressure_operator", "jacobi_pcg",
    "mass_and_convection", "dye_implicit_step",
]

TOL = 1e-6
H = 1.0
L = 1.0


def _chunks(n, workers):
    """[0, n) in `workers` contiguous ranges."""
    b = np.linspace(0, n, workers + 1).astype(np.int64)
    return [(int(b[k]), int(b[k + 1])) for k in range(workers) if b[k + 1] > b[k]]


def _threaded(fn, n, workers):
    """fn(lo, hi) over `workers` contiguous ranges of [0, n) on a thread pool (numpy's array kernels
    release the GIL); returns the per-range results in range order.  workers <= 1: one call."""
    if workers <= 1:
        return [fn(0, n)]
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(workers) as ex:
        return list(ex.map(lambda r: fn(*r), _chunks(n, workers)))


# ----------------------------------------------------------------------------- mesh I/O
def read_node(path, dtype=np.float64):
    """StokesColor.py:54-78 (fp64) / poisson.py:27-56 (fp32, :40): header N, then N lines id x y marker."""
    with open(path) as f:
        n = int(f.readline().split()[0])
        X = np.zeros((n, 2), dtype=dtype)
        mk = np.zeros(n, dtype=np.int32)
        for _ in range(n):
            t = f.readline().split()
            i = int(t[0]) - 1
            X[i, 0] = float(t[1])
            X[i, 1] = float(t[2])
            if int(t[3]) != 0:
                mk[i] = int(t[3])
    return X, mk


def read_ele(path):
    """StokesColor.py:82-95: header T, then T lines id a b c (1-based -> 0-based)."""
    with open(path) as f:
        nt = int(f.readline().split()[0])
        T = np.zeros((nt, 3), dtype=np.int32)
        for k in range(nt):
            t = f.readline().split()
            T[k] = [int(t[1]) - 1, int(t[2]) - 1, int(t[3]) - 1]
    return T


def read_poly(path):
    """poisson.py:76-97: skip line 1, segment header, segments (1-based) + optional marker."""
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


def find_boundary_pairs(X, L=1.0, tol=TOL):
    """StokesColor.py:169-203: each left (x~0) node -> right (x~L) node of nearest y (1-D KDTree)."""
    left = np.where(np.abs(X[:, 0]) < tol)[0]
    right = np.where(np.abs(X[:, 0] - L) < tol)[0]
    if len(left) == 0 or len(right) == 0:
        return np.zeros((0, 2), dtype=np.int64)
    # scipy KDTree (leafsize 10), one query per left node, as the reference: exact y-ties
    # (mesh2.1 node 260) resolve by the tree's traversal order, which this reproduces.
    tree = KDTree(X[right, 1].reshape(-1, 1))
    j = [int(tree.query([X[i, 1]])[1]) for i in left]
    return np.stack([left, right[j]], 1).astype(np.int64)


def filter_wall_pairs(X, pairs, tol=TOL, H=H):
    """StokesColor.py:449-457 / poisson.py:242-246: drop pairs whose master lies on y=0 or y=H."""
    if len(pairs) == 0:
        return pairs
    y = X[pairs[:, 0], 1]
    keep = ~((np.abs(y - 0.0) < tol) | (np.abs(y - H) < tol))
    return pairs[keep]


def boundary_sets(X, mk, tol=TOL, H=H):
    """StokesColor.py:461-464: wall (y=0|H), inner (marker 2), dirichlet, interior."""
    wall = np.where(np.isclose(X[:, 1], 0.0, atol=tol) | np.isclose(X[:, 1], H, atol=tol))[0]
    inner = np.where(mk == 2)[0]
    dirichlet = np.union1d(wall, inner)
    interior = np.setdiff1d(np.arange(X.shape[0]), dirichlet)
    return wall, inner, dirichlet, interior


# ----------------------------------------------------------------------------- assembly
def _xy(X, T):
    return (X[T[:, 0], 0], X[T[:, 0], 1], X[T[:, 1], 0], X[T[:, 1], 1], X[T[:, 2], 0], X[T[:, 2], 1])


def _scatter_csr(N, rows, cols, vals):
    """Accumulate (rows, cols, vals) in the given order into CSR (sorted columns)."""
    key = rows.astype(np.int64) * N + cols
    uk, inv = np.unique(key, return_inverse=True)
    data = np.zeros(len(uk))
    np.add.at(data, inv, vals)
    r = (uk // N).astype(np.int64)
    c = (uk % N).astype(np.int64)
    return sp.csr_matrix((data, (r, c)), shape=(N, N))


def stiffness(X, T):
    """StokesColor.py:98-128: K_ij += (b_i b_j + c_i c_j) / (2|det|), skip |det| < 1e-14 (fp64)."""
    x1, y1, x2, y2, x3, y3 = _xy(X, T)
    det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2)
    ok = np.abs(det) >= 1e-14
    yd = np.stack([y2 - y3, y3 - y1, y1 - y2], 1)
    xd = np.stack([x3 - x2, x1 - x3, x2 - x1], 1)
    den = 2 * np.abs(det)
    vals = (yd[:, :, None] * yd[:, None, :] + xd[:, :, None] * xd[:, None, :]) / den[:, None, None]
    rows = np.repeat(T[:, :, None], 3, 2)
    cols = np.repeat(T[:, None, :], 3, 1)
    s = ok
    return _scatter_csr(X.shape[0], rows[s].ravel(), cols[s].ravel(), vals[s].ravel())


def lumped_mass(X, T):
    """StokesColor.py:266-284: M_i = sum over triangles of area/3 (no degenerate skip)."""
    x1, y1, x2, y2, x3, y3 = _xy(X, T)
    det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2)
    a3 = 0.5 * np.abs(det) / 3.0
    M = np.zeros(X.shape[0])
    np.add.at(M, T.ravel(), np.repeat(a3, 3))
    return M


def div_area_sum(X, T):
    """StokesColor.py:139-165: area_sum as accumulated by calculate_divergence (|det| >= 1e-14 only)."""
    x1, y1, x2, y2, x3, y3 = _xy(X, T)
    det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2)
    ok = np.abs(det) >= 1e-14
    a3 = np.where(ok, 0.5 * np.abs(det) / 3.0, 0.0)
    S = np.zeros(X.shape[0])
    np.add.at(S, T[ok].ravel(), np.repeat(a3[ok], 3))
    return S


def divergence(X, T, u, workers=1):
    """StokesColor.py:130-165 calculate_divergence: lumped nodal divergence / (area_sum + 1e-12).
    workers > 1 (the CPU baseline's timing leg only): the triangle loop in contiguous chunks on threads,
    per-chunk node sums added in chunk order -- the same arithmetic, node sums associated differently."""
    if workers > 1:
        parts = _threaded(lambda a, b: _divergence_sums(X, T[a:b], u), T.shape[0], workers)
        ds = sum(p[0] for p in parts)
        asum = sum(p[1] for p in parts)
        return ds / (asum + 1e-12)
    ds, asum = _divergence_sums(X, T, u)
    return ds / (asum + 1e-12)


def _divergence_sums(X, T, u):
    x1, y1, x2, y2, x3, y3 = _xy(X, T)
    det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2)
    ok = np.abs(det) >= 1e-14
    inv = 1.0 / np.where(ok, det, 1.0)
    area = 0.5 * np.abs(det)
    ux, uy = u[:, 0], u[:, 1]
    a, b, c = T[:, 0], T[:, 1], T[:, 2]
    dux = (ux[a] * (y2 - y3) + ux[b] * (y3 - y1) + ux[c] * (y1 - y2)) * inv
    duy = (uy[a] * (x3 - x2) + uy[b] * (x1 - x3) + uy[c] * (x2 - x1)) * inv
    lump = (dux + duy) * (area / 3.0)
    ds = np.zeros(X.shape[0])
    asum = np.zeros(X.shape[0])
    # reference order: for each triangle, for p in tri: div_sum[p] += lump; area_sum[p] += area/3
    np.add.at(ds, T[ok].ravel(), np.repeat(lump[ok], 3))
    np.add.at(asum, T[ok].ravel(), np.repeat((area / 3.0)[ok], 3))
    return ds, asum


def gradient(X, T, p, workers=1):
    """StokesColor.py:224-263 calculate_gradiant: lumped nodal gradient / (area_sum + 1e-12).
    workers > 1: as divergence."""
    if workers > 1:
        parts = _threaded(lambda a, b: _gradient_sums(X, T[a:b], p), T.shape[0], workers)
        sx, sy, asum = (sum(q[k] for q in parts) for k in range(3))
    else:
        sx, sy, asum = _gradient_sums(X, T, p)
    return sx / (asum + 1e-12), sy / (asum + 1e-12)


def _gradient_sums(X, T, p):
    x1, y1, x2, y2, x3, y3 = _xy(X, T)
    det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2)
    ok = np.abs(det) >= 1e-14
    inv = 1.0 / np.where(ok, det, 1.0)
    area = 0.5 * np.abs(det)
    a, b, c = T[:, 0], T[:, 1], T[:, 2]
    gx = ((y2 - y3) * inv) * p[a] + ((y3 - y1) * inv) * p[b] + ((y1 - y2) * inv) * p[c]
    gy = ((x3 - x2) * inv) * p[a] + ((x1 - x3) * inv) * p[b] + ((x2 - x1) * inv) * p[c]
    a3 = area / 3.0
    sx = np.zeros(X.shape[0])
    sy = np.zeros(X.shape[0])
    asum = np.zeros(X.shape[0])
    idx = T[ok].ravel()
    np.add.at(sx, idx, np.repeat((gx * a3)[ok], 3))
    np.add.at(sy, idx, np.repeat((gy * a3)[ok], 3))
    np.add.at(asum, idx, np.repeat(a3[ok], 3))
    return sx, sy, asum


def fem_system_fp32(X32, T, g_source):
    """poisson.py:100-146 buildFemSystem with fp32 coordinates (:40): fp32 element arithmetic,
    fp64 accumulation in triangle order, exact-zero skip, load g(centroid)*area/3; returns (A, -b)."""
    assert X32.dtype == np.float32
    x1, y1, x2, y2, x3, y3 = _xy(X32, T)
    det = x1 * y2 - x1 * y3 - x2 * y1 + x2 * y3 + x3 * y1 - x3 * y2
    ok = det != 0
    yd = np.stack([y2 - y3, y3 - y1, y1 - y2], 1)
    xd = np.stack([x3 - x2, x1 - x3, x2 - x1], 1)
    den = np.float32(2.0) * det
    vals = (yd[:, :, None] * yd[:, None, :] + xd[:, :, None] * xd[:, None, :]) / den[:, None, None]
    assert vals.dtype == np.float32
    rows = np.repeat(T[:, :, None], 3, 2)
    cols = np.repeat(T[:, None, :], 3, 1)
    N = X32.shape[0]
    A = _scatter_csr(N, rows[ok].ravel(), cols[ok].ravel(), vals[ok].astype(np.float64).ravel())
    area = np.float32(0.5) * det
    if callable(g_source):
        g = g_source((x1 + x2 + x3) / np.float32(3), (y1 + y2 + y3) / np.float32(3))
    else:
        g = np.full(len(T), g_source)
    s = g * (area / np.float32(3))
    b = np.zeros(N)
    np.add.at(b, T[ok].ravel(), np.repeat(s[ok].astype(np.float64), 3))
    return A, -b


def apply_periodic_rowmerge(A, b, pairs):
    """poisson.py:187-213: row m += row s; b_m += b_s; row s <- e_s - e_m; b_s = 0 (sequential)."""
    A = A.tolil(copy=True)
    b = b.copy()
    for m, s in pairs:
        A[m, :] = A[m, :] + A[s, :]
        b[m] += b[s]
        A[s, :] = 0.0
        A[s, s] = 1.0
        A[s, m] = -1.0
        b[s] = 0.0
    return A.tocsr(), b


def _dirichlet_mask32(X32, mk, tol=TOL, H=H):
    y = X32[:, 1]
    wall = (np.abs(y - np.float32(0.0)) < tol) | (np.abs(y - np.float32(H)) < tol)
    inner = mk == 2
    return wall, inner


def apply_dirichlet_rows(A, b, X32, mk, wall_value=1.0, inner_value=0.0):
    """poisson.py:258-278: Dirichlet rows only (columns kept); inner -> 0.0, wall -> 1.0."""
    wall, inner = _dirichlet_mask32(X32, mk)
    A = A.tolil(copy=True)
    b = b.copy()
    for i in np.where(wall | inner)[0]:
        A[i, :] = 0.0
        A[i, i] = 1.0
        b[i] = inner_value if inner[i] else wall_value
    return A.tocsr(), b


def poisson_literal(X32, mk, T):
    """poisson.py:218-285 end to end: fp32 assembly, filtered row-merge, Dirichlet rows, direct solve."""
    pairs = find_boundary_pairs(X32)
    A, b = fem_system_fp32(X32, T, lambda x, y: 50 * np.sin(3 * y))
    A, b = apply_periodic_rowmerge(A, b, filter_wall_pairs(X32, pairs))
    A, b = apply_dirichlet_rows(A, b, X32, mk)
    return spla.spsolve(A.tocsc(), b), A, b


class HeatLiteral:
    """heatEq.py:219-325: A <- I + DT*A (Poisson operator incl. BC rows); u <- A^-1 u; then
    reapply_periodic_u with the UNFILTERED pairs (:298-301) and reapply_dirchlect_u (:282-295)."""

    def __init__(self, X32, mk, T, dt=0.02):
        _, A, _ = poisson_literal(X32, mk, T)
        N = X32.shape[0]
        self.A = (sp.identity(N, format="csr") + dt * A).tocsc()
        self.lu = spla.splu(self.A)
        self.pairs = find_boundary_pairs(X32)
        self.wall, self.inner = _dirichlet_mask32(X32, mk)
        self.N = N

    def bc(self, u):
        for m, s in self.pairs:
            u[s] = u[m]
        u[self.inner] = 0.0
        u[self.wall & ~self.inner] = 1.0
        return u

    def initial(self):
        return self.bc(np.zeros(self.N))

    def step(self, u):
        return self.bc(self.lu.solve(u))


# ----------------------------------------------------------------------------- Stokes pieces
def squirmer_bc(X, inner, B1, B2, center=(0.5, 0.5)):
    """StokesColor.py:405-427 makeDirBCU inner-body values (theta = arctan2, v_t = B1 sin + B2 sin 2)."""
    rx = X[inner, 0] - center[0]
    ry = X[inner, 1] - center[1]
    th = np.arctan2(ry, rx)
    vt = B1 * np.sin(th) + B2 * np.sin(2 * th)
    return np.stack([vt * -np.sin(th), vt * np.cos(th)], 1)


def make_dir_bcu(u, wall, inner, inner_vals):
    """StokesColor.py:405-427: walls <- (0,0), then inner squirmer values."""
    u[wall] = 0.0
    u[inner] = inner_vals
    return u


def make_per_bcu(u, pairs):
    """StokesColor.py:429-431: u[slave] = u[master], sequentially in pair order."""
    for m, s in pairs:
        u[s] = u[m]
    return u


def visc_matrix(K, dt, nu, dirichlet):
    """StokesColor.py:471-475: I + dt*nu*K with Dirichlet rows AND columns zeroed, diagonal 1."""
    N = K.shape[0]
    A = (sp.identity(N, format="csr") + dt * nu * K).tolil()
    D = np.zeros(N, dtype=bool)
    D[dirichlet] = True
    A = A.tocsr()
    A = sp.diags((~D).astype(float)) @ A @ sp.diags((~D).astype(float)) + sp.diags(D.astype(float))
    return A.tocsr()


class PressureSolver:
    """Well-posed restatement of StokesColor.py:478-479 + :554-555.

    Reference: A_p = K/(M+1e-12) plus a 1e10 periodic penalty, solved by dense LU -- singular
    (pure Neumann) with an inconsistent RHS.  Restatement: multiply row i by (M_i+1e-12),
    merge each periodic slave into its master (P^T K P), project the RHS onto the range
    (zero sum over free dofs), solve for the zero-mean pressure, copy master -> slave."""

    def __init__(self, K, M, pairs):
        N = K.shape[0]
        self.N = N
        self.M = M
        self.pairs = pairs
        dof = np.arange(N)
        for m, s in pairs:
            dof[s] = m
        slaves = np.zeros(N, dtype=bool)
        slaves[pairs[:, 1]] = True
        if len(pairs) and len(np.unique(pairs[:, 1])) != len(pairs):
            raise ValueError("duplicate periodic slave")
        self.free = np.where(~slaves)[0]
        pos = -np.ones(N, dtype=np.int64)
        pos[self.free] = np.arange(len(self.free))
        self.pos = pos[dof]
        P = sp.csr_matrix((np.ones(N), (np.arange(N), self.pos)), shape=(N, len(self.free)))
        self.P = P
        self.Kr = (P.T @ K @ P).tocsc()
        self.lu = spla.splu(self.Kr[1:, 1:].tocsc())

    def rhs(self, b_p):
        r = (self.M + 1e-12) * b_p
        rr = self.P.T @ r
        return rr - rr.mean()

    def solve(self, b_p):
        rr = self.rhs(b_p)
        x = np.zeros(len(self.free))
        x[1:] = self.lu.solve(rr[1:])
        x -= x.mean()
        return self.P @ x


def centroids(X, T):
    """StokesColor.py:321: np.mean(nodes[triangles], axis=1)."""
    return np.mean(X[T], axis=1)


def sl_advect(c, u, dt, X, T, tree=None, k=10, workers=1):
    """StokesColor.py:347-389 advect_semilagrange with PointLocator.find (:314-345): back-trace,
    x wrapped mod 1, y clamped to [1e-12, 1-1e-12], first of the k nearest centroids whose
    barycentric weights are all >= 0, periodic-dx interpolation, not found -> keep c[n]."""
    if tree is None:
        tree = KDTree(centroids(X, T))
    xb = np.remainder(X[:, 0] - dt * u[:, 0] * 1.0, 1.0)
    yb = X[:, 1] - dt * u[:, 1] * 1.0
    yb = np.where(yb < 0.0, 1e-12, yb)
    yb = np.where(yb > 1.0, 1.0 - 1e-12, yb)
    # workers > 1 (the CPU baseline's timing leg): the k-NN query and the per-node tests on threads --
    # every node is independent, so the result is the same
    _, idx = tree.query(np.stack([xb, yb], 1), k=k, workers=workers)
    N = X.shape[0]
    found = -np.ones(N, dtype=np.int64)

    def first_hit(a, b):
        xq, yq, fd = xb[a:b], yb[a:b], found[a:b]
        for kk in range(k):
            t = idx[a:b, kk]
            i, j, l_ = T[t, 0], T[t, 1], T[t, 2]
            x1, y1, x2, y2, x3, y3 = X[i, 0], X[i, 1], X[j, 0], X[j, 1], X[l_, 0], X[l_, 1]
            det = (x2 - x1) * (y3 - y1) - (x3 - x1) * (y2 - y1)
            okd = np.abs(det) >= 1e-14
            sd = np.where(okd, det, 1.0)
            w1 = ((x2 - xq) * (y3 - yq) - (x3 - xq) * (y2 - yq)) / sd
            w2 = ((x3 - xq) * (y1 - yq) - (x1 - xq) * (y3 - yq)) / sd
            w3 = 1.0 - w1 - w2
            hit = okd & (w1 >= 0.0) & (w2 >= 0.0) & (w3 >= 0.0) & (fd < 0)
            fd[hit] = t[hit]

    _threaded(first_hit, N, workers)

    def dx(a, b):
        d = a - b
        d = np.where(d > 0.5, d - 1.0, d)
        return np.where(d < -0.5, d + 1.0, d)

    out = c.copy()
    f = found >= 0
    t = found[f]
    i, j, l_ = T[t, 0], T[t, 1], T[t, 2]
    xf, yf = xb[f], yb[f]
    x1, y1, x2, y2, x3, y3 = X[i, 0], X[i, 1], X[j, 0], X[j, 1], X[l_, 0], X[l_, 1]
    det = dx(x2, x1) * (y3 - y1) - dx(x3, x1) * (y2 - y1)
    w1 = (dx(x2, xf) * (y3 - yf) - dx(x3, xf) * (y2 - yf)) / det
    w2 = (dx(x3, xf) * (y1 - yf) - dx(x1, xf) * (y3 - yf)) / det
    w3 = 1.0 - w1 - w2
    out[f] = w1 * c[i] + w2 * c[j] + w3 * c[l_]
    return out, ~f


def mixing_index(c, mass, mask=None):
    """StokesColor.py:391-403: Danckwerts I = Var_w(c) / (mu (1-mu) + 1e-16); returns (I, mu, var)."""
    if mask is not None:
        c = c[mask]
        mass = mass[mask]
    W = mass.sum()
    mu = (mass @ c) / W
    var = (mass @ (c - mu) ** 2) / W
    return var / (mu * (1 - mu) + 1e-16), mu, var


# ----------------------------------------------------------------------------- tracers
def plane_coefficients(X, T, z):
    """matplotlib 3.10 Triangulation::calculate_plane_coefficients (C++, used by
    LinearTriInterpolator at StokesFood.py:482-486): normal = (p1-p0) x (p2-p0) in (x,y,z);
    a = -n_x/n_z, b = -n_y/n_z, c = n.p0/n_z; z(x,y) = a x + b y + c."""
    p0 = np.stack([X[T[:, 0], 0], X[T[:, 0], 1], z[T[:, 0]]], 1)
    s1 = np.stack([X[T[:, 1], 0], X[T[:, 1], 1], z[T[:, 1]]], 1) - p0
    s2 = np.stack([X[T[:, 2], 0], X[T[:, 2], 1], z[T[:, 2]]], 1) - p0
    nx = s1[:, 1] * s2[:, 2] - s1[:, 2] * s2[:, 1]
    ny = s1[:, 2] * s2[:, 0] - s1[:, 0] * s2[:, 2]
    nz = s1[:, 0] * s2[:, 1] - s1[:, 1] * s2[:, 0]
    dot = nx * p0[:, 0] + ny * p0[:, 1] + nz * p0[:, 2]
    return np.stack([-nx / nz, -ny / nz, dot / nz], 1)


def locate_bary(X, T, px, py):
    """Point location (matplotlib TrapezoidMapTriFinder semantics: containing triangle or -1);
    restated as a brute-force orientation test, lowest triangle index on shared edges."""
    x1, y1, x2, y2, x3, y3 = _xy(X, T)
    out = -np.ones(len(px), dtype=np.int64)
    for n in range(len(px)):
        x, y = px[n], py[n]
        if not (np.isfinite(x) and np.isfinite(y)):
            continue
        o1 = (x2 - x1) * (y - y1) - (y2 - y1) * (x - x1)
        o2 = (x3 - x2) * (y - y2) - (y3 - y2) * (x - x2)
        o3 = (x1 - x3) * (y - y3) - (y1 - y3) * (x - x3)
        hit = np.where((o1 >= 0) & (o2 >= 0) & (o3 >= 0))[0]
        if len(hit):
            out[n] = hit[0]
    return out


def tracer_init(squirmer_radius=0.25, center=(0.5, 0.5), density=25, L=1.0, H=1.0):
    """StokesFood.py:420-430: 25x25 grid in [0.05, 0.95]^2, drop points with r <= radius."""
    xx = np.linspace(0.05, L - 0.05, density)
    yy = np.linspace(0.05, H - 0.05, density)
    gx, gy = np.meshgrid(xx, yy)
    pts = np.vstack([gx.ravel(), gy.ravel()]).T
    d = np.linalg.norm(pts - np.array(center), axis=1)
    return pts[d > squirmer_radius].copy()


def tracer_step(pts, status, u, dt, X, T, capture=0.28, center=(0.5, 0.5)):
    """StokesFood.py:482-499: linear interpolation of u (NaN outside the mesh), forward Euler,
    x mod 1, sticky capture when |x - c| <= capture radius."""
    tri = locate_bary(X, T, pts[:, 0], pts[:, 1])
    vel = np.full((len(pts), 2), np.nan)
    ok = tri >= 0
    for d in range(2):
        pc = plane_coefficients(X, T, u[:, d])[tri[ok]]
        vel[ok, d] = pc[:, 0] * pts[ok, 0] + pc[:, 1] * pts[ok, 1] + pc[:, 2]
    pts = pts.copy()
    pts[:, 0] += vel[:, 0] * dt
    pts[:, 1] += vel[:, 1] * dt
    pts[:, 0] = np.mod(pts[:, 0], 1.0)
    dist = np.linalg.norm(pts - np.array(center), axis=1)
    status = status.copy()
    status[np.where(dist <= capture)[0]] = 1
    return pts, status


# ----------------------------------------------------------------------------- full Stokes step
class StokesRef:
    """StokesColor.py:437-586 / StokesFood.py:357-505: one operator-split step with the
    symmetric-merged pressure (PressureSolver).  ``scheme`` 'color' advects dye, 'food' moves tracers."""

    def __init__(self, X, mk, T, dt, nu, B1, B2, scheme="color", workers=1):
        # workers > 1: bench.py's CPU-baseline timing leg (element loops, SL and the two viscous solves on
        # threads); the parity tests use the default single-threaded path
        self.workers = workers
        self.X, self.mk, self.T = X, mk, T
        self.N = X.shape[0]
        self.dt, self.nu = dt, nu
        pairs = filter_wall_pairs(X, find_boundary_pairs(X))
        self.pairs = pairs
        self.wall, self.inner, self.dirichlet, self.interior = boundary_sets(X, mk)
        self.K = stiffness(X, T)
        self.M = lumped_mass(X, T)
        self.inner_vals = squirmer_bc(X, self.inner, B1, B2)
        self.Av = visc_matrix(self.K, dt, nu, self.dirichlet)
        self.lu_v = spla.splu(self.Av.tocsc())
        self.ps = PressureSolver(self.K, self.M, pairs)
        self.scheme = scheme
        self.tree = KDTree(centroids(X, T))
        self.mask_inner = np.where(mk == 0)[0]

    def initial(self):
        u = np.zeros((self.N, 2))
        make_dir_bcu(u, self.wall, self.inner, self.inner_vals)
        c = np.zeros(self.N)
        c[self.X[:, 0] < 0.5] = 1.0
        return u, c

    def bc(self, u):
        make_per_bcu(u, self.pairs)
        make_dir_bcu(u, self.wall, self.inner, self.inner_vals)
        return u

    def step(self, u, c=None, tracers=None, status=None):
        X, T, dt = self.X, self.T, self.dt
        W = self.workers
        us = np.zeros_like(u)
        if W > 1:
            cols = _threaded(lambda a, b: self.lu_v.solve(u[:, a] + dt * 0.0), 2, 2)
            us[:, 0], us[:, 1] = cols[0], cols[1]
        else:
            us[:, 0] = self.lu_v.solve(u[:, 0] + dt * 0.0)
            us[:, 1] = self.lu_v.solve(u[:, 1] + dt * 0.0)
        self.bc(us)
        div_s = divergence(X, T, us, W)
        p = self.ps.solve(-(1.0 / dt) * div_s)
        gx, gy = gradient(X, T, p, W)
        un = np.empty_like(u)
        un[:, 0] = us[:, 0] - dt * gx
        un[:, 1] = us[:, 1] - dt * gy
        self.bc(un)
        div_u = divergence(X, T, un, W)
        p2 = self.ps.solve(-(1.0 / dt) * div_u)
        g2x, g2y = gradient(X, T, p2, W)
        I = self.interior
        un[I, 0] -= dt * g2x[I]
        un[I, 1] -= dt * g2y[I]
        fdiv = divergence(X, T, un, W)
        out = dict(u_star=us, div_u_star=div_s, p=p, div_u=div_u, p2=p2, final_div=fdiv, u=un)
        if c is not None:
            c2, nf = sl_advect(c, un, dt, X, T, self.tree, workers=W)
            out["c"] = c2
            out["sl_notfound"] = nf
            out["mixing"] = mixing_index(c2, self.M, mask=self.mask_inner)
        if tracers is not None:
            out["tracers"], out["status"] = tracer_step(tracers, status, un, dt, X, T)
        return out


# ----------------------------------------------------------------------------- implicit dye variant
def mass_and_convection(X, T, u):
    """build_mass_and_convection (StokesColor.py:286-312 = good_visualization.py:348-374): the
    consistent mass M_ij += area/12 (2 on the diagonal) and the convection matrix
    C_ij += area/3 <u_c, grad_j> with u_c the triangle's vertex mean and grad_j scaled by 1/(2|det|)
    (|det|, not the signed det), skipping |det| < 1e-14; accumulated in triangle order."""
    x1, y1, x2, y2, x3, y3 = _xy(X, T)
    det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2)
    ok = np.abs(det) >= 1e-14
    area = 0.5 * np.abs(det)
    fac = np.where(np.eye(3, dtype=bool), 2.0, 1.0)
    mv = (area / 12.0)[:, None, None] * fac[None]
    uc = ((u[T[:, 0]] + u[T[:, 1]]) + u[T[:, 2]]) / 3.0
    den = 2 * np.abs(det)
    gx = np.stack([y2 - y3, y3 - y1, y1 - y2], 1) / den[:, None]
    gy = np.stack([x3 - x2, x1 - x3, x2 - x1], 1) / den[:, None]
    dot = uc[:, 0:1] * gx + uc[:, 1:2] * gy            # (T, 3): <u_c, grad_j>
    cv = np.repeat(((area / 3)[:, None] * dot)[:, None, :], 3, 1)  # row i, column j
    rows = np.repeat(T[:, :, None], 3, 2)[ok].ravel()
    cols = np.repeat(T[:, None, :], 3, 1)[ok].ravel()
    N = X.shape[0]
    return _scatter_csr(N, rows, cols, mv[ok].ravel()), _scatter_csr(N, rows, cols, cv[ok].ravel())


def dye_implicit_step(c, u, X, T, pairs, dt, D, K=None, merged=True):
    """One step of the implicit FEM dye advection-diffusion (good_visualization.py:700-718):
    A = M + dt (C_u + D K) + diag(G), G = dt M_lumped div(u) with G[slave] = G[master],
    rhs = M c, c = A^-1 rhs, c[slave] = c[master].  The reference makes M and A periodic with a
    1e10 penalty (apply_periodic_bc, :179-194, on M at :592 and on A at :711); merged=True solves
    the penalty's limit exactly -- slave columns folded into the masters, the pair rows summed --
    merged=False the literal penalised system (sparse LU)."""
    N = X.shape[0]
    M, C = mass_and_convection(X, T, u)
    K = stiffness(X, T) if K is None else K
    G = dt * (lumped_mass(X, T) * divergence(X, T, u))
    pairs = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    G[pairs[:, 1]] = G[pairs[:, 0]]
    A = (M + dt * (C + D * K) + sp.diags(G)).tocsr()
    if merged:
        # the limit: the summed pair rows (penalties cancel) and 2 pen (x_m - x_s) = pen (c_m - c_s) + O(1),
        # i.e. x_s = x_m - delta_s with delta_s = (c_m - c_s) / 2 (zero once c is periodic); with
        # x = P y - delta:  P^T A P y = P^T (M c + A delta), and the final copy leaves c = P y
        dof = np.arange(N)
        dof[pairs[:, 1]] = pairs[:, 0]
        P = sp.csr_matrix((np.ones(N), (np.arange(N), dof)), shape=(N, N))
        Am = (P.T @ A @ P).tolil()
        Am[pairs[:, 1], pairs[:, 1]] = 1.0
        delta = np.zeros(N)
        delta[pairs[:, 1]] = (c[pairs[:, 0]] - c[pairs[:, 1]]) / 2
        b = P.T @ (M @ c + A @ delta)
        b[pairs[:, 1]] = c[pairs[:, 0]]
        x = spla.spsolve(Am.tocsc(), b)
    else:
        pen = 1.0e10
        Pn = sp.lil_matrix((N, N))
        for m, s in pairs:
            Pn[m, m] += pen
            Pn[s, s] += pen
            Pn[m, s] -= pen
            Pn[s, m] -= pen
        Mp = (M + Pn).tocsr()
        x = spla.spsolve((Mp + dt * (C + D * K) + sp.diags(G) + Pn).tocsc(), Mp @ c)
    x = np.asarray(x)
    x[pairs[:, 1]] = x[pairs[:, 0]]
    return x


# ----------------------------------------------------------------------------- CPU baseline helpers
def pressure_operator(K, pairs):
    """P^T K P of PressureSolver without the factorisation (node numbering, slave rows identity)."""
    N = K.shape[0]
    dof = np.arange(N)
    dof[pairs[:, 1]] = pairs[:, 0]
    P = sp.csr_matrix((np.ones(N), (np.arange(N), dof)), shape=(N, N))
    A = (P.T @ K @ P).tolil()
    A[pairs[:, 1], pairs[:, 1]] = 1.0
    return A.tocsr()


def jacobi_pcg(A, b, x0, iters):
    """`iters` iterations of Jacobi-preconditioned CG (the algorithm of the HIP solver), scipy CSR."""
    dinv = 1.0 / A.diagonal()
    x = x0.copy()
    r = b - A @ x
    z = dinv * r
    p = z.copy()
    rz = r @ z
    for _ in range(iters):
        q = A @ p
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        z = dinv * r
        rz2 = r @ z
        p = z + (rz2 / rz) * p
        rz = rz2
    return x, float(np.sqrt(r @ r))
