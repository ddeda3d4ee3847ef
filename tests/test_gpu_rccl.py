"""RCCL on the library stream, on the one-GPU box.

The multi-rank data path -- all-reduced CG dots (the dot products inside the np.linalg.solve calls of
StokesColor.py:544-545, 555, 569), broadcasts into the replicated coarse levels, the dye range
exchange -- runs through `Comm`.  The LocalComm tests cover its call sequence with W ranks on one
GPU; RCCL itself refuses two ranks on one device.  A ONE-rank context created from a real
ncclGetUniqueId gets an RCCL communicator and takes every multi-rank code path through it, so the
RCCL linkage, the stream ordering of its collectives and the API use are executed here before the
driver's 8-GPU run.
"""
import ctypes as ct
import os

import numpy as np
import pytest

from conftest import has_gpu, load_pkg

pytestmark = pytest.mark.gpu

pf = load_pkg()
from importlib import import_module  # noqa: E402

L = import_module("puc-fluidsimulation-project_amd._lib")
S = import_module("puc-fluidsimulation-project_amd.solver")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not has_gpu():
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    # single-node bootstrap: the loopback interface is always there
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")


def unique_id():
    uid = (ct.c_uint8 * 128)()
    L.check(L.lib().pucfem_rccl_unique_id(uid))
    return bytes(uid)


@pytest.mark.timeout(300)
def test_rccl_one_rank_selftest_and_steps(monkeypatch):
    """RCCL communicator of one rank: the all-reduce / ring send-recv self-test on the library stream,
    then 6 StokesColor steps on L3 at the production settings through the multi-rank code path, equal
    to the plain single-rank run in the same PCG form (the multi-rank pressure solves run the single-reduction
    Chronopoulos-Gear PCG: PUCFEM_CGCG=1 puts the reference run on it)."""
    mesh = pf.load_mesh("fine", refine=3)
    tol = S.Tolerances.production()
    sim = S.StokesSimulation(mesh, S.SquirmerBC(), 0.05, "color", 0, tol, dist=(0, 1, unique_id()))
    assert sim.ctx.comm_info()["backend"] == "rccl"
    t = sim.ctx.comm_selftest()
    assert t["backend"] == "rccl" and t["sum_err"] == 0 and t["max_err"] == 0 and t["recv_err"] == 0, t
    monkeypatch.setenv("PUCFEM_CGCG", "1")
    ref = S.StokesSimulation(mesh, S.SquirmerBC(), 0.05, "color", 0, tol)
    assert ref.ctx.comm_info()["backend"] is None
    for k in range(6):
        a, b = sim.step(1)[0], ref.step(1)[0]
        assert (a.it_visc, a.it_p, a.it_p2) == (b.it_visc, b.it_p, b.it_p2), k
        assert np.abs(sim.u - ref.u).max() <= 1e-12, k
        assert np.abs(sim.c - ref.c).max() <= 1e-12, k
        assert abs(a.mix_var - b.mix_var) <= 1e-14, k
    sim.close()
    ref.close()


@pytest.mark.timeout(300)
def test_rccl_one_rank_food_tracers(monkeypatch):
    """The StokesFood tracer exchange (one all-reduce of 3 x 488 values per step) through RCCL."""
    mesh = pf.load_mesh("fine", refine=2)
    tol = S.Tolerances.production()
    bc = S.SquirmerBC(B2=-5.0, nu=1.0)
    sim = S.StokesSimulation(mesh, bc, 0.01, "food", 0, tol, dist=(0, 1, unique_id()))
    monkeypatch.setenv("PUCFEM_CGCG", "1")  # (the multi-rank PCG form)
    ref = S.StokesSimulation(mesh, bc, 0.01, "food", 0, tol)
    sa, sb = sim.step(5), ref.step(5)
    assert sim.ctx.comm_info()["tracer_allreduce_values"] == 3 * 488
    np.testing.assert_allclose(sim.u, ref.u, rtol=0, atol=1e-12)
    tr, trr = sim.tracers, ref.tracers
    assert np.array_equal(np.isnan(tr), np.isnan(trr))
    ok = ~np.isnan(trr)
    assert np.abs(tr[ok] - trr[ok]).max() <= 1e-12
    assert [s.eaten for s in sa] == [s.eaten for s in sb]
    sim.close()
    ref.close()
