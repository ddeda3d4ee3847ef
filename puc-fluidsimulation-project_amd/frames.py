"""Frame / field export for visualisation (scripts/good_visualization2.py:536-571,
:724-747).  Host side only: the fields are copied off the GPU at the recorded steps.

The reference keeps a copy of the dye and the velocity every ``frame_interval`` (50) steps, then
animates a gouraud ``tripcolor`` of the dye (magma, [0, 1]) under a ``quiver`` of every ``skip``-th
node's velocity, titled "Fluid Simulation - Step k", and saves it with ffmpeg at 20 fps, 150 dpi.
``FrameRecorder`` does the same around a ``StokesSimulation``; ``render`` writes the animation with
ffmpeg when it is installed, else an animated GIF (Pillow) or a PNG sequence; ``save_npz`` /
``load_npz`` keep the raw frames and ``write_vtk`` writes one frame as a legacy VTK unstructured grid
(ParaView / VisIt), which needs no plotting stack at all.
"""
from __future__ import annotations

import os
import shutil

import numpy as np


class FrameRecorder:
    """Record (step, dye, velocity) every `interval` steps of a simulation (fp32 copies by default,
    half the host memory of the reference's fp64 lists)."""

    def __init__(self, mesh, interval=50, dtype=np.float32):
        self.mesh = mesh
        self.interval = int(interval)
        self.dtype = dtype
        self.steps: list[int] = []
        self.dye: list[np.ndarray] = []
        self.vel: list[np.ndarray] = []

    def record(self, step, c, u):
        self.steps.append(int(step))
        self.dye.append(np.array(c, dtype=self.dtype, copy=True) if c is not None else None)
        self.vel.append(np.array(u, dtype=self.dtype, copy=True))

    def run(self, sim, steps):
        """Step `sim` (a StokesSimulation) `steps` times, recording the state after every step whose
        index is a multiple of `interval` (good_visualization2.py:724).  Steps between two recorded
        ones run in one call (no host synchronisation per step).  Returns the per-step stats."""
        stats = []
        end = sim.step_count + steps
        while sim.step_count < end:
            k0 = sim.step_count
            r = -(-k0 // self.interval) * self.interval  # next recorded step index
            n = min(end, r + 1) - k0
            stats += sim.step(n)
            if sim.step_count - 1 == r:
                self.record(r, sim.c if sim.scheme == "color" else None, sim.u)
        return stats

    def __len__(self):
        return len(self.steps)


def save_npz(rec: FrameRecorder, path):
    d = dict(steps=np.array(rec.steps), coords=rec.mesh.coords, triangles=rec.mesh.triangles,
             vel=np.stack(rec.vel) if rec.vel else np.zeros((0, rec.mesh.N, 2)))
    if rec.dye and rec.dye[0] is not None:
        d["dye"] = np.stack(rec.dye)
    np.savez_compressed(path, **d)


def load_npz(path):
    d = np.load(path)
    return {k: d[k] for k in d.files}


def write_vtk(path, coords, triangles, point_data: dict):
    """One frame as a legacy binary VTK unstructured grid: triangles (cell type 5), point scalars
    (1-component fields) and vectors (2-component fields, z = 0)."""
    X = np.asarray(coords, dtype=np.float64)
    T = np.asarray(triangles, dtype=np.int64)
    N, M = len(X), len(T)
    with open(path, "wb") as f:
        f.write(b"# vtk DataFile Version 3.0\npucfem frame\nBINARY\nDATASET UNSTRUCTURED_GRID\n")
        f.write(f"POINTS {N} double\n".encode())
        pts = np.zeros((N, 3), dtype=">f8")
        pts[:, :2] = X
        f.write(pts.tobytes())
        f.write(f"\nCELLS {M} {4 * M}\n".encode())
        cells = np.empty((M, 4), dtype=">i4")
        cells[:, 0] = 3
        cells[:, 1:] = T
        f.write(cells.tobytes())
        f.write(f"\nCELL_TYPES {M}\n".encode())
        f.write(np.full(M, 5, dtype=">i4").tobytes())
        f.write(f"\nPOINT_DATA {N}\n".encode())
        for name, a in point_data.items():
            a = np.asarray(a, dtype=np.float64)
            if a.ndim == 1:
                f.write(f"SCALARS {name} double 1\nLOOKUP_TABLE default\n".encode())
                f.write(a.astype(">f8").tobytes())
            else:
                v = np.zeros((N, 3), dtype=">f8")
                v[:, :2] = a
                f.write(f"VECTORS {name} double\n".encode())
                f.write(v.tobytes())
            f.write(b"\n")


def read_vtk_header(path):
    """(n_points, n_cells, field names) of a file written by write_vtk (tests, tools)."""
    with open(path, "rb") as f:
        data = f.read()
    n_pts = n_cells = None
    names = []
    i = 0
    while i < len(data):
        j = data.find(b"\n", i)
        line = data[i:j if j >= 0 else len(data)]
        tok = line.split()
        step = 0
        if tok[:1] == [b"POINTS"]:
            n_pts = int(tok[1])
            step = n_pts * 24
        elif tok[:1] == [b"CELLS"]:
            n_cells = int(tok[1])
            step = int(tok[2]) * 4
        elif tok[:1] == [b"CELL_TYPES"]:
            step = int(tok[1]) * 4
        elif tok[:1] == [b"SCALARS"]:
            names.append(tok[1].decode())
            j = data.find(b"\n", j + 1)  # LOOKUP_TABLE line
            step = n_pts * 8
        elif tok[:1] == [b"VECTORS"]:
            names.append(tok[1].decode())
            step = n_pts * 24
        if j < 0:
            break
        i = j + 1 + step
    return n_pts, n_cells, names


def render(rec: FrameRecorder, out, fps=20, dpi=150, skip=None):
    """Animate the recorded frames as the reference does (tripcolor of the dye + quiver of the
    velocity, good_visualization2.py:536-571).  out ending in .mp4 uses ffmpeg (if installed), .gif
    Pillow; a directory name writes frame_00000.png ...  Returns the written path(s)."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    import matplotlib.tri as mtri
    from matplotlib import animation

    X, T = rec.mesh.coords, rec.mesh.triangles
    skip = skip or max(1, len(X) // 1500)
    tri = mtri.Triangulation(X[:, 0], X[:, 1], T)
    fig, ax = plt.subplots(figsize=(8, 8))
    dye0 = rec.dye[0] if rec.dye and rec.dye[0] is not None else np.zeros(len(X))
    tpc = ax.tripcolor(tri, dye0, shading="gouraud", cmap="magma", vmin=0, vmax=1.0)
    fig.colorbar(tpc, ax=ax, label="Dye concentration")
    qv = ax.quiver(X[::skip, 0], X[::skip, 1], rec.vel[0][::skip, 0], rec.vel[0][::skip, 1], color="white", scale=20.0)
    ax.set_aspect("equal")
    ax.set_xlim(0, 1)
    ax.set_ylim(0, 1)
    title = ax.set_title(f"Fluid Simulation - Step {rec.steps[0]}")

    def update(i):
        if rec.dye[i] is not None:
            tpc.set_array(rec.dye[i])
        qv.set_UVC(rec.vel[i][::skip, 0], rec.vel[i][::skip, 1])
        title.set_text(f"Fluid Simulation - Step {rec.steps[i]}")
        return tpc, qv, title

    out = str(out)
    if out.endswith(".mp4") and shutil.which("ffmpeg"):
        ani = animation.FuncAnimation(fig, update, frames=len(rec), interval=50, blit=False)
        ani.save(out, writer="ffmpeg", fps=fps, dpi=dpi)
        written = [out]
    elif out.endswith(".gif") or out.endswith(".mp4"):
        if out.endswith(".mp4"):  # no ffmpeg on this machine
            out = out[:-4] + ".gif"
        ani = animation.FuncAnimation(fig, update, frames=len(rec), interval=50, blit=False)
        ani.save(out, writer=animation.PillowWriter(fps=fps), dpi=dpi // 2)
        written = [out]
    else:
        os.makedirs(out, exist_ok=True)
        written = []
        for i in range(len(rec)):
            update(i)
            p = os.path.join(out, f"frame_{i:05d}.png")
            fig.savefig(p, dpi=dpi // 2)
            written.append(p)
    plt.close(fig)
    return written
