"""Reference-named entry points (StokesColor.py / poisson.py function names and signatures).

The hot-path functions (calculate_divergence, calculate_gradiant, advect_semilagrange, the two
np.linalg.solve call sites) run on the GPU through a context cached per mesh.  The assembly
functions return the C++ host-assembled operator (dense for small meshes, as the reference's
np.zeros((N, N)) matrices; scipy CSR above DENSE_MAX nodes).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .mesh import Mesh, boundary_sets
from .solver import Context, SquirmerBC, Tolerances, stokes_setup

DENSE_MAX = 8192
_cache: dict = {}


def _key(nodes, triangles):
    n = np.ascontiguousarray(nodes, dtype=np.float64)
    t = np.ascontiguousarray(triangles, dtype=np.int32)
    return (n.shape, t.shape, hash(n.tobytes()), hash(t.tobytes())), n, t


def context_for(nodes, triangles, dt=0.05, nu=0.1, bc: SquirmerBC | None = None, device=0):
    """A single-GPU Stokes context for this mesh (cached by content)."""
    (k, n, t) = _key(nodes, triangles)
    k = k + (dt, nu, None if bc is None else (bc.B1, bc.B2))
    ctx = _cache.get(k)
    if ctx is None:
        mesh = Mesh(n, np.zeros(len(n), dtype=np.int32), t)
        ctx = Context(device)
        ctx.upload(mesh)
        ctx.build("color", dt, nu, Tolerances())
        _cache[k] = ctx
    return ctx


def _stokes_context(mesh: Mesh, dt, nu, bc: SquirmerBC, device=0):
    # the Dirichlet set and values depend on the markers and the squirmer geometry, not only on the mesh
    k = ("stokes", mesh.N, mesh.T, hash(mesh.coords.tobytes()), hash(mesh.triangles.tobytes()),
         hash(np.ascontiguousarray(mesh.markers).tobytes()), dt, nu, bc.B1, bc.B2, tuple(bc.center),
         tuple(bc.outer_value), bc.capture_radius, bc.squirmer_radius)
    ctx = _cache.get(k)
    if ctx is None:
        ctx = Context(device)
        ctx.upload(mesh)
        pairs, nodes, vals = stokes_setup(mesh, bc)
        ctx.set_pairs(0, pairs)
        ctx.set_pairs(1, pairs)
        ctx.set_dirichlet(nodes, vals)
        ctx.build("color", dt, nu, Tolerances(), capture=bc.capture_radius, center=bc.center)
        _cache[k] = ctx
    return ctx


# The reference's functions read module globals (nodes_coords, triangles, pairs, B1, B2, ...,
# StokesColor.py:359,369,405-431); set_globals() plays that role for the shims that keep the
# reference's short signatures (advect_semilagrange(c, u, DT), makeDirBCU(u), makePerBCU(u)).
_globals: dict = {}


def set_globals(mesh: Mesh, bc: SquirmerBC | None = None):
    """Bind the mesh (and squirmer parameters) the reference-signature shims act on."""
    _globals.clear()
    _globals.update(mesh=mesh, bc=bc or SquirmerBC())


def _mesh_or_global(mesh):
    if mesh is None:
        mesh = _globals.get("mesh")
    if mesh is None:
        raise ValueError("no mesh: pass mesh= or call set_globals(mesh) first (the reference's module globals)")
    return mesh


def makeDirBCU(u, mesh: Mesh | None = None, bc: SquirmerBC | None = None):
    """StokesColor.py:405-427 in place on u (N,2): walls to 0, squirmer surface to the tangential
    squirmer velocity, through the device's boundary kernel."""
    mesh = _mesh_or_global(mesh)
    _apply_bc(u, mesh, bc or _globals.get("bc") or SquirmerBC(), 2)


def makePerBCU(u, mesh: Mesh | None = None, bc: SquirmerBC | None = None):
    """StokesColor.py:429-431 in place on u (N,2): u[slave] = u[master] for the filtered pairs."""
    mesh = _mesh_or_global(mesh)
    _apply_bc(u, mesh, bc or _globals.get("bc") or SquirmerBC(), 1)


def _apply_bc(u, mesh, bc, which):
    if not (isinstance(u, np.ndarray) and u.dtype == np.float64 and u.flags.c_contiguous and u.shape == (mesh.N, 2)):
        raise TypeError("u must be a C-contiguous float64 array of shape (N, 2) (modified in place)")
    ctx = _stokes_context(mesh, 0.05, bc.nu, bc)
    _lib.check(ctx.L.pucfem_apply_bc(ctx.h, which, _lib.dptr(u)), ctx.h)


def mixing_index(c, mass, mask=None, mesh: Mesh | None = None):
    """StokesColor.py:391-403: (I, mu, var) of c weighted by `mass` over `mask` (None: every node), on
    the device.  The reference's c[mask], mass[mask] becomes the node weights w = mass on the mask and 0
    elsewhere (an index mask with repeats counts a node repeatedly, a boolean mask selects), so any
    weights and mask the reference accepts are accepted here."""
    mesh = _mesh_or_global(mesh)
    c = np.ascontiguousarray(c, dtype=np.float64)
    mass = np.asarray(mass, dtype=np.float64)
    if c.shape != (mesh.N,) or mass.shape != (mesh.N,):
        raise ValueError(f"mixing_index: c and mass must have shape ({mesh.N},)")
    if mask is None:
        w = mass
    else:
        m = np.asarray(mask)
        if m.dtype == bool:
            if m.shape != (mesh.N,):
                raise ValueError(f"mixing_index: a boolean mask must have shape ({mesh.N},)")
            w = np.where(m, mass, 0.0)
        else:
            m = m.astype(np.int64).ravel()
            m = np.where(m < 0, m + mesh.N, m)  # numpy's negative indices
            if m.size and (m.min() < 0 or m.max() >= mesh.N):
                raise IndexError("mixing_index: mask index out of range")
            w = np.bincount(m, minlength=mesh.N).astype(np.float64) * mass
    ctx = _stokes_context(mesh, 0.05, 0.1, _globals.get("bc") or SquirmerBC())
    out = np.zeros(3)
    w = np.ascontiguousarray(w, dtype=np.float64)
    _lib.check(ctx.L.pucfem_mixing_index_w(ctx.h, _lib.dptr(c), _lib.dptr(w), _lib.dptr(out)), ctx.h)
    return float(out[0]), float(out[1]), float(out[2])


def calculate_divergence(nodes, triangles, u_star):
    """StokesColor.py:130-165 on the GPU: (N,) lumped nodal divergence."""
    ctx = context_for(nodes, triangles)
    return ctx.apply(_lib.OP_DIV, np.asarray(u_star, dtype=np.float64).reshape(-1, 2), (len(nodes),))


def calculate_gradiant(nodes, triangles, p_scalar):
    """StokesColor.py:224-263 on the GPU: (grad_px, grad_py)."""
    ctx = context_for(nodes, triangles)
    g = ctx.apply(_lib.OP_GRAD, np.asarray(p_scalar, dtype=np.float64), (len(nodes), 2))
    return g[:, 0].copy(), g[:, 1].copy()


def advect_semilagrange(c, u, DT, nodes=None, triangles=None):
    """StokesColor.py:347-389 on the GPU, in place on c like the reference (c[:] = c_new).
    advect_semilagrange(c, u, DT) as in the reference acts on the set_globals() mesh.
    Returns the not-found mask (nodes that kept c[n])."""
    if nodes is None or triangles is None:
        m = _mesh_or_global(None)
        nodes, triangles = m.coords, m.triangles
    ctx = context_for(nodes, triangles)
    cin = np.ascontiguousarray(c, dtype=np.float64)
    uu = np.ascontiguousarray(u, dtype=np.float64).reshape(-1, 2)
    out = np.zeros_like(cin)
    nf = np.zeros(len(cin), dtype=np.int32)
    _lib.check(ctx.L.pucfem_sl_advect(ctx.h, _lib.dptr(cin), _lib.dptr(uu), float(DT), _lib.dptr(out),
                                      _lib.iptr(nf)), ctx.h)
    c[:] = out
    return nf.astype(bool)


def buildStiffnessMatrix(nodes, triangles, g_source=1.0):
    """StokesColor.py:98-128: (A, -B) with B = 0 (the reference never fills it)."""
    ctx = context_for(nodes, triangles)
    A = ctx.host_csr(_lib.OP_K)
    return (A.toarray() if len(nodes) <= DENSE_MAX else A), np.zeros(len(nodes))


def buildLumpedMassMatrix(nodes_coords, triangles):
    """StokesColor.py:266-284 (host setup): M_i = sum of area/3 over incident triangles."""
    X = np.asarray(nodes_coords, dtype=np.float64)
    T = np.asarray(triangles)
    x1, y1, x2, y2, x3, y3 = X[T[:, 0], 0], X[T[:, 0], 1], X[T[:, 1], 0], X[T[:, 1], 1], X[T[:, 2], 0], X[T[:, 2], 1]
    det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2)
    M = np.zeros(len(X))
    np.add.at(M, T.ravel(), np.repeat(0.5 * np.abs(det) / 3.0, 3))
    return M


def mixing_index_host(mesh: Mesh, c):
    """mixing_index (StokesColor.py:391-403) of a host field over marker==0 nodes: used once for
    the initial (I0, mu0, var0) normaliser of the printed progress (StokesColor.py:497)."""
    M = buildLumpedMassMatrix(mesh.coords, mesh.triangles)
    mask = np.where(mesh.markers == 0)[0]
    cc, mm = c[mask], M[mask]
    W = mm.sum()
    mu = (mm @ cc) / W
    var = (mm @ (cc - mu) ** 2) / W
    return var / (mu * (1 - mu) + 1e-16), mu, var


def solve_viscous(mesh: Mesh, rhs, dt=0.05, nu=0.1, bc: SquirmerBC | None = None, rtol=1e-13):
    """The np.linalg.solve(A_visc, rhs) call sites (StokesColor.py:544-545) for both components."""
    ctx = _stokes_context(mesh, dt, nu, bc or SquirmerBC(nu=nu))
    x, it = ctx.solve(_lib.OP_VISC, np.asarray(rhs, dtype=np.float64).reshape(-1, 2), rtol=rtol)
    return x


def solve_pressure(mesh: Mesh, b_p, dt=0.05, nu=0.1, bc: SquirmerBC | None = None, rtol=1e-12):
    """The np.linalg.solve(A_pressure, b_p) call sites (StokesColor.py:555, :569), restated as the
    well-posed periodic-merged system; returns the zero-mean pressure."""
    ctx = _stokes_context(mesh, dt, nu, bc or SquirmerBC(nu=nu))
    x, it = ctx.solve(_lib.OP_PRES, np.asarray(b_p, dtype=np.float64), rtol=rtol)
    return x


def _dye_context(mesh: Mesh, dt, D, device=0):
    k = ("dye", mesh.N, mesh.T, hash(mesh.coords.tobytes()), hash(mesh.triangles.tobytes()), dt, D)
    ctx = _cache.get(k)
    if ctx is None:
        bc = SquirmerBC()
        ctx = Context(device)
        ctx.upload(mesh)
        pairs, nodes, vals = stokes_setup(mesh, bc)
        ctx.set_pairs(0, pairs)
        ctx.set_pairs(1, pairs)
        ctx.set_dirichlet(nodes, vals)
        ctx.build("color", dt, bc.nu, Tolerances(dye="implicit", dye_diffusivity=D))
        _cache[k] = ctx
    return ctx


def dye_implicit_step(c, u, mesh: Mesh, dt=0.05, D=1e-3):
    """One implicit FEM dye advection-diffusion step (scripts/good_visualization.py:700-718) on the
    GPU: A = M + dt (C_u + D K) + diag(dt M_lumped div u), c <- A^-1 M c with the periodic pairs
    merged exactly (the reference's 1e10 penalty in its limit), then c[slave] = c[master].
    Returns (c_new, BiCGStab iterations)."""
    ctx = _dye_context(mesh, dt, D)
    cin = np.ascontiguousarray(c, dtype=np.float64)
    uu = np.ascontiguousarray(u, dtype=np.float64).reshape(-1, 2)
    out = np.zeros_like(cin)
    it = np.zeros(1, dtype=np.int32)
    _lib.check(ctx.L.pucfem_dye_step(ctx.h, _lib.dptr(cin), _lib.dptr(uu), _lib.dptr(out), _lib.iptr(it)), ctx.h)
    return out, int(it[0])


def build_mass_and_convection_mass(mesh: Mesh):
    """The M of build_mass_and_convection (StokesColor.py:286-312): the consistent mass, host-assembled
    (scipy CSR, caller numbering); C_u is assembled on the device inside every implicit dye step."""
    ctx = _dye_context(mesh, 0.05, 1e-3)
    return ctx.host_csr(_lib.OP_MCONS)


def clear_cache():
    for c in _cache.values():
        c.close()
    _cache.clear()
