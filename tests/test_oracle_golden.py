"""Pin the CPU oracle (oracle/fem_ref.py) against fixtures produced by running the reference.

Bit-exact where the oracle restates the reference's arithmetic in the same order
(assembly, lumping, divergence, BCs, semi-Lagrangian advection); within stated
tolerances where the reference delegates to LAPACK / matplotlib C++.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import oracle as O
from conftest import REFERENCE

MESHES = ["mesh1", "mesh21", "fine"]
FILES = {
    "mesh1": "code/mesh/mesh.1",
    "mesh21": "resources/mesh2.1",
    "fine": "resources/mesh_fine.1",
}


def dense(ij, v, N):
    A = np.zeros((N, N))
    A[ij[0], ij[1]] = v
    return A


@pytest.mark.parametrize("m", MESHES)
def test_reader_on_reference_files(m, golden):
    g = golden(m)
    base = os.path.join(REFERENCE, FILES[m])
    if not os.path.exists(base + ".node"):
        pytest.skip("reference mesh files not present (GPU box)")
    X, mk = O.read_node(base + ".node")
    X32, _ = O.read_node(base + ".node", np.float32)
    T = O.read_ele(base + ".ele")
    assert np.array_equal(X, g["coords64"]) and X.dtype == np.float64
    assert np.array_equal(X32, g["coords32"]) and X32.dtype == np.float32
    assert np.array_equal(mk, g["markers"]) and mk.dtype == np.int32
    assert np.array_equal(T, g["tris"]) and T.dtype == np.int32
    seg, sm = O.read_poly(base + ".poly")
    assert np.array_equal(seg, g["poly_segments"]) and np.array_equal(sm, g["poly_markers"])


@pytest.mark.parametrize("m", MESHES)
def test_pairs(m, golden):
    g = golden(m)
    X = g["coords64"]
    p = O.find_boundary_pairs(X)
    assert np.array_equal(p, g["pairs_all"])
    assert np.array_equal(O.filter_wall_pairs(X, p), g["pairs"])
    assert np.array_equal(O.find_boundary_pairs(g["coords32"]), g["pairs32_all"])


@pytest.mark.parametrize("m", MESHES)
def test_assembly_bitexact(m, golden):
    g = golden(m)
    X, T = g["coords64"], g["tris"]
    N = X.shape[0]
    K = O.stiffness(X, T).toarray()
    assert np.array_equal(K, dense(g["K_ij"], g["K_v"], N))
    assert np.array_equal(O.lumped_mass(X, T), g["M"])
    A, b = O.fem_system_fp32(g["coords32"], T, lambda x, y: 50 * np.sin(3 * y))
    assert np.array_equal(A.toarray(), dense(g["Apois_ij"], g["Apois_v"], N))
    assert np.array_equal(b, g["bpois"])


@pytest.mark.parametrize("m", MESHES)
def test_div_grad(m, golden):
    g = golden(m)
    X, T = g["coords64"], g["tris"]
    assert np.array_equal(O.divergence(X, T, g["u_rand"]), g["div_rand"])
    assert np.array_equal(O.divergence(X, T, np.stack([2 * X[:, 0], 3 * X[:, 1]], 1)), g["div_lin"])
    gx, gy = O.gradient(X, T, g["p_rand"])
    np.testing.assert_allclose(np.stack([gx, gy], 1), g["grad_rand"], rtol=0, atol=1e-12)
    gx, gy = O.gradient(X, T, 2 * X[:, 0] + 3 * X[:, 1])
    np.testing.assert_allclose(np.stack([gx, gy], 1), g["grad_lin"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("m", MESHES)
def test_bc_and_visc(m, golden):
    g = golden(m)
    X, T, mk = g["coords64"], g["tris"], g["markers"]
    wall, inner, dirichlet, interior = O.boundary_sets(X, mk)
    assert np.array_equal(wall, g["wall"]) and np.array_equal(interior, g["interior"])
    for tag, B2 in (("neutral", 0.0), ("pusher", -5.0), ("puller", 5.0)):
        u = np.full((X.shape[0], 2), 7.0)
        O.make_dir_bcu(u, wall, inner, O.squirmer_bc(X, inner, -2.0, B2))
        assert np.array_equal(u, g[f"dirbc_{tag}"])
    K = O.stiffness(X, T)
    import scipy.sparse.linalg as spla

    for tag, dt, nu in (("color", 0.05, 0.1), ("food", 0.01, 1.0)):
        A = O.visc_matrix(K, dt, nu, dirichlet)
        x = spla.spsolve(A.tocsc(), g["u_rand"][:, 0])
        np.testing.assert_allclose(x, g[f"visc_{tag}_x"], rtol=0, atol=1e-13)


@pytest.mark.parametrize("m", MESHES)
def test_semilagrange_bitexact(m, golden):
    g = golden(m)
    X, T = g["coords64"], g["tris"]
    for tag, dt in (("small", 0.05), ("large", 0.2)):
        c, nf = O.sl_advect(g["c0"], g["u_swirl"], dt, X, T)
        assert np.array_equal(nf, g[f"sl_{tag}_notfound"])
        assert np.array_equal(c, g[f"sl_{tag}"])
    I, mu, var = O.mixing_index(g["sl_small"], g["M"], mask=np.where(g["markers"] == 0)[0])
    np.testing.assert_allclose([I, mu, var], g["mixing_sl_small"], rtol=1e-14)


@pytest.mark.parametrize("m", MESHES)
def test_tracers(m, golden):
    g = golden(m)
    X, T = g["coords64"], g["tris"]
    pts = O.tracer_init()
    assert np.array_equal(pts, g["tracer0"])
    st = np.zeros(len(pts), dtype=int)
    for _ in range(10):
        pts, st = O.tracer_step(pts, st, g["u_swirl"], 0.01, X, T)
    np.testing.assert_allclose(pts, g["tracer10"], rtol=0, atol=1e-12)
    assert np.array_equal(np.isnan(pts), np.isnan(g["tracer10"]))
    assert np.array_equal(st, g["tracer10_status"])


@pytest.mark.parametrize("m", MESHES)
def test_poisson_literal(m, golden):
    g = golden(m)
    f, _, _ = O.poisson_literal(g["coords32"], g["markers"], g["tris"])
    np.testing.assert_allclose(f, g["poisson_f"], rtol=0, atol=1e-10)


KNOWN = {  # SURVEY.md §4 known answers (reference run headless)
    "poisson_sum": {"mesh1": -11.930071025687944, "mesh21": -25.089913100232543, "fine": -47.1538503108591},
    "heat600_sum": {"mesh1": 122.74951817118082, "fine": 297.6348323970126},
}


@pytest.mark.parametrize("m", MESHES)
def test_golden_matches_survey_known_answers(m, golden):
    g = golden(m)
    assert abs(g["poisson_f"].sum() - KNOWN["poisson_sum"][m]) < 1e-10
    if m in KNOWN["heat600_sum"]:
        assert abs(g["heat_u600"].sum() - KNOWN["heat600_sum"][m]) < 1e-9


@pytest.mark.parametrize("m", MESHES)
def test_heat_literal(m, golden):
    g = golden(m)
    h = O.HeatLiteral(g["coords32"], g["markers"], g["tris"])
    u = h.initial()
    for k in range(1, 601):
        u = h.step(u)
        if k in (1, 10, 600):
            np.testing.assert_allclose(u, g[f"heat_u{k}"], rtol=0, atol=1e-10)


@pytest.mark.parametrize("m", ["mesh1", "fine"])
def test_stokes_first_steps(m, golden):
    """Contract (i) on the pressure-free parts of step 0, contract (iii) on the rest."""
    g = golden(m)
    S = O.StokesRef(g["coords64"], g["markers"], g["tris"], 0.05, 0.1, -2.0, 0.0, "color")
    u, c = S.initial()
    out = S.step(u, c)
    np.testing.assert_allclose(out["u_star"], g["color_s0_u_star"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(out["div_u_star"], g["color_s0_div_u_star"], rtol=0, atol=1e-10)
    # pressure-dependent outputs: the reference's LU noise floor
    np.testing.assert_allclose(out["u"], g["color_s0_u"], rtol=0, atol=1e-2)
    for k in (1, 2):
        out = S.step(out["u"], out["c"])
        np.testing.assert_allclose(out["u"], g[f"color_s{k}_u"], rtol=0, atol=1e-2)
    np.testing.assert_allclose(out["c"], g["color_s2_c"], rtol=0, atol=1e-2)
