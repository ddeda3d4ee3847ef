"""The Python boundary on the GPU (SURVEY.md §8 b): the north-star ``solve(mesh, bc, dt, steps,
scheme)`` surface on all four schemes and the reference-named shims with the reference's own
signatures (StokesColor.py:347, :391-431), against the goldens the reference produced.

Tolerances as tests/test_gpu_parity.py: Poisson / heat 1e-10 vs the reference; Stokes vs the
literal reference at its pressure noise floor (1e-2 in u); the boundary
conditions, mixing index and semi-Lagrangian step bit-exact or at rounding.
"""
import numpy as np

import oracle as O
import pytest

from conftest import has_gpu, load_pkg

pytestmark = pytest.mark.gpu

pf = load_pkg()


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not has_gpu():
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")


def test_solve_color(golden):
    g = golden("mesh1")
    mesh = pf.load_mesh("mesh1")
    lines = []
    res = pf.solve(mesh, steps=3, scheme="color", log=lines.append)
    assert res.u.shape == (mesh.N, 2) and res.c.shape == (mesh.N,) and len(res.stats) == 3
    assert np.abs(res.u - g["color_s2_u"]).max() < 1e-2
    assert np.abs(res.c - g["color_s2_c"]).max() < 1e-2
    # the reference's per-step line (StokesColor.py:583-586): same fields, values at the noise floor
    for mine, ref in zip(lines, g["color_log"]):
        a, b = mine.split(", "), str(ref).split(", ")
        assert [x.split(":")[0].split("=")[0] for x in a] == [x.split(":")[0].split("=")[0] for x in b]
        assert a[0] == b[0]


def test_solve_food(golden):
    g = golden("mesh1")
    mesh = pf.load_mesh("mesh1")
    lines = []
    res = pf.solve(mesh, pf.SquirmerBC(B2=-5.0, nu=1.0), steps=3, scheme="food", log=lines.append)
    assert np.abs(res.u - g["food_s2_u"]).max() < 1e-2
    ref = g["food_s2_tracer_points"]
    assert np.array_equal(np.isnan(res.tracers), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.abs(res.tracers[ok] - ref[ok]).max() < 1e-2
    assert np.array_equal(res.tracer_status.astype(int), g["food_s2_tracer_status"])
    assert lines[-1].startswith("Step: 2, Div(u*): ") and "Eaten (Red): " in lines[-1]


@pytest.mark.parametrize("m", ["mesh1", "fine"])
def test_solve_heat_and_poisson(m, golden):
    g = golden(m)
    mesh = pf.load_mesh(m)
    res = pf.solve(mesh, steps=10, scheme="heat")
    np.testing.assert_allclose(res.scalar, g["heat_u10"], rtol=0, atol=1e-10)
    res = pf.solve(mesh, scheme="poisson")
    np.testing.assert_allclose(res.scalar, g["poisson_f"], rtol=0, atol=1e-10)


@pytest.mark.parametrize("tag,B2", [("neutral", 0.0), ("pusher", -5.0), ("puller", 5.0)])
def test_makeDirBCU_makePerBCU(tag, B2, golden):
    """makeDirBCU(u) on u = 7 everywhere = the reference's output (StokesColor.py:405-427), exactly;
    makePerBCU(u) copies master -> slave over the filtered pairs (StokesColor.py:429-431)."""
    g = golden("fine")
    mesh = pf.load_mesh("fine")
    pf.set_globals(mesh, pf.SquirmerBC(B2=B2))
    u = np.full((mesh.N, 2), 7.0)
    pf.makeDirBCU(u)
    np.testing.assert_array_equal(u, g[f"dirbc_{tag}"])
    u = np.random.default_rng(3).standard_normal((mesh.N, 2))
    want = u.copy()
    for m_, s_ in g["pairs"]:
        want[s_] = want[m_]
    pf.makePerBCU(u)
    np.testing.assert_array_equal(u, want)


def test_mixing_index_and_short_semilagrange_signature(golden):
    """mixing_index(c, M, mask) and advect_semilagrange(c, u, DT) with the reference's signatures
    (module globals bound by set_globals) = the reference's outputs."""
    g = golden("fine")
    mesh = pf.load_mesh("fine")
    pf.set_globals(mesh)
    c = g["c0"].copy()
    pf.advect_semilagrange(c, g["u_swirl"], 0.05)
    np.testing.assert_array_equal(c, g["sl_small"])
    M = pf.buildLumpedMassMatrix(mesh.coords, mesh.triangles)
    I, mu, var = pf.mixing_index(c, M, mask=np.where(mesh.markers == 0)[0])
    np.testing.assert_allclose([I, mu, var], g["mixing_sl_small"], rtol=1e-12, atol=0)
    # any weights and masks the reference accepts (StokesColor.py:397-403): no mask (every node), a
    # boolean mask, other weights, an index mask with repeats -- against the oracle's restatement
    rng = np.random.default_rng(3)
    w = rng.uniform(0.5, 2.0, mesh.N)
    idx = rng.integers(0, mesh.N, mesh.N // 3)
    for mass, mask in ((M, None), (2 * M, mesh.markers == 0), (w, None), (w, idx)):
        got = pf.mixing_index(c, mass, mask=mask)
        np.testing.assert_allclose(got, O.mixing_index(c, mass, mask=mask), rtol=1e-12, atol=1e-15)
    with pytest.raises(ValueError):
        pf.mixing_index(c[:-1], M)


def test_frame_recorder_on_a_run(tmp_path):
    """Frame export around a real StokesColor run (good_visualization2.py:724): frames after steps
    0, 50, 100; the last one is the simulation's final state; a VTK of it carries the same fields."""
    mesh = pf.load_mesh("mesh1")
    sim = pf.StokesSimulation(mesh)
    rec = pf.FrameRecorder(mesh, interval=50, dtype=np.float64)
    st = rec.run(sim, 101)
    assert len(st) == 101 and rec.steps == [0, 50, 100]
    np.testing.assert_array_equal(rec.dye[-1], sim.c)
    np.testing.assert_array_equal(rec.vel[-1], sim.u)
    pf.write_vtk(str(tmp_path / "last.vtk"), mesh.coords, mesh.triangles, {"dye": sim.c, "velocity": sim.u})
    sim.close()
