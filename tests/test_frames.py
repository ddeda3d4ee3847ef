"""Frame / field export (scripts/good_visualization2.py:536-571, :724-747): the
recorder's step selection, the .npz round trip, the VTK writer and the renderer (PNG sequence and
animated GIF -- ffmpeg, which the reference's mp4 needs, is not installed here)."""
import os

import numpy as np

from conftest import load_pkg

pf = load_pkg()
from importlib import import_module  # noqa: E402

F = import_module("puc-fluidsimulation-project_amd.frames")


class FakeSim:
    """The StokesSimulation surface the recorder uses, with fields that encode the step index."""

    scheme = "color"

    def __init__(self, mesh):
        self.mesh = mesh
        self.step_count = 0
        self.calls = []

    def step(self, n):
        self.calls.append(n)
        self.step_count += n
        return [object()] * n

    @property
    def c(self):
        return np.full(self.mesh.N, float(self.step_count - 1)) / 1000.0

    @property
    def u(self):
        return np.full((self.mesh.N, 2), float(self.step_count - 1))


def test_recorder_steps_like_the_reference():
    """Frames after steps 0, 50, 100, ... (step % frame_interval == 0), intermediate steps batched."""
    mesh = pf.load_mesh("mesh1")
    sim = FakeSim(mesh)
    rec = pf.FrameRecorder(mesh, interval=50)
    st = rec.run(sim, 120)
    assert len(st) == 120 and sim.step_count == 120
    assert rec.steps == [0, 50, 100]
    assert sim.calls == [1, 50, 50, 19]
    for k, c, u in zip(rec.steps, rec.dye, rec.vel):
        assert np.all(c == np.float32(k / 1000.0)) and np.all(u == k)
    # continuing a run keeps the global step index
    rec.run(sim, 31)
    assert rec.steps == [0, 50, 100, 150]


def test_npz_vtk_and_render(tmp_path):
    mesh = pf.load_mesh("mesh1")
    X = mesh.coords
    rec = pf.FrameRecorder(mesh, interval=1)
    for k in range(3):
        rec.record(k, 0.5 + 0.5 * np.sin(3 * X[:, 0] + k), np.stack([np.cos(X[:, 1] + k), np.sin(X[:, 0])], 1))
    p = str(tmp_path / "frames.npz")
    pf.save_npz(rec, p)
    d = pf.load_npz(p)
    assert d["dye"].shape == (3, mesh.N) and d["vel"].shape == (3, mesh.N, 2)
    np.testing.assert_array_equal(d["steps"], [0, 1, 2])
    np.testing.assert_array_equal(d["triangles"], mesh.triangles)
    v = str(tmp_path / "f.vtk")
    pf.write_vtk(v, X, mesh.triangles, {"dye": d["dye"][1], "velocity": d["vel"][1]})
    n, m, names = F.read_vtk_header(v)
    assert (n, m, names) == (mesh.N, mesh.T, ["dye", "velocity"])
    # binary payload: the point coordinates and the dye values as written (big-endian fp64)
    raw = open(v, "rb").read()
    i = raw.index(b"POINTS") + len(f"POINTS {mesh.N} double\n")
    pts = np.frombuffer(raw[i:i + 24 * mesh.N], dtype=">f8").reshape(-1, 3)
    np.testing.assert_array_equal(pts[:, :2], X)
    pngs = pf.render(rec, str(tmp_path / "png"))
    assert len(pngs) == 3 and all(os.path.getsize(q) > 1000 for q in pngs)
    gif = pf.render(rec, str(tmp_path / "anim.mp4"), fps=5, dpi=60)
    assert len(gif) == 1 and os.path.getsize(gif[0]) > 1000
