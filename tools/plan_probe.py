"""Host-only: rank R's multigrid plans and deep-halo flags of a W-rank run (PUCFEM_PLAN_EMULATE; no GPU).
  python tools/plan_probe.py LEVEL W [RANK] [MG_REP_NODES]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg  # noqa: E402

level, world = int(sys.argv[1]), int(sys.argv[2])
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rep = int(sys.argv[4]) if len(sys.argv) > 4 else 0
os.environ["PUCFEM_PLAN_EMULATE"] = f"{rank},{world}"
os.environ["PUCFEM_DEEP_REPORT"] = "1"
pf = load_pkg()
S = __import__("importlib").import_module("puc-fluidsimulation-project_amd.solver")
L = __import__("importlib").import_module("puc-fluidsimulation-project_amd._lib")
mesh = pf.load_mesh("fine", refine=level)
ctx = S.Context(L.HOST_ONLY)
ctx.upload(mesh)
pairs, nodes, vals = S.stokes_setup(mesh, S.SquirmerBC())
ctx.set_pairs(0, pairs)
ctx.set_pairs(1, pairs)
ctx.set_dirichlet(nodes, vals)
ctx.set_hierarchy(mesh.base, mesh.levels)
ctx.build("color", 0.05, 0.1, S.Tolerances.production(mg_rep_nodes=rep))
print(ctx.info())
