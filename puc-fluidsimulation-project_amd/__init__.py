"""pucfem-mi355x: the MI355X (gfx950) hot path of TobiasHoffmannP/PUC-Fluidsimulation-Project.

Host side: Python (this package) -> ctypes -> libpucfem.so (C ABI, include/pucfem.h) -> HIP
kernels for CDNA4.  Entry points mirror the reference (code/StokesColor.py, StokesFood.py,
poisson.py, heatEq.py): the mesh loaders readNode / readEle / readPoly, the reference-named
operators, and ``solve(mesh, bc, dt, steps, scheme)``.

The directory name contains hyphens, so import it with
``importlib.import_module("puc-fluidsimulation-project_amd")``.
"""
from ._lib import PucfemError, device_count, lib as _load_library  # noqa: F401
from .mesh import (Mesh, boundary_sets, filter_wall_pairs, find_boundary_pairs, load_mesh, readEle,  # noqa: F401
                   readNode, readPoly, writeEle, writeNode, writePoly)
from .ops import (advect_semilagrange, buildLumpedMassMatrix, buildStiffnessMatrix, calculate_divergence,  # noqa: F401
                  build_mass_and_convection_mass, calculate_gradiant, dye_implicit_step, makeDirBCU, makePerBCU,
                  mixing_index, set_globals, solve_pressure, solve_viscous)
from .solver import (Context, HeatSimulation, Result, SquirmerBC, StokesSimulation, Tolerances,  # noqa: F401
                     poisson_solve, solve, squirmer_values)
from .frames import FrameRecorder, load_npz, render, save_npz, write_vtk  # noqa: F401
from .tracers import tracer_init  # noqa: F401

__version__ = "0.1.0"
