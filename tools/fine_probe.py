"""mesh_fine (BASELINE configs[2]) StokesColor steps for a kernel trace of the small-mesh path: 20 warm-up steps
(the first captures the step into a hipGraph), then STEPS timed steps in one pucfem_step call.
  python tools/fine_probe.py [STEPS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg  # noqa: E402

pf = load_pkg()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
mesh = pf.load_mesh("fine")
sim = pf.StokesSimulation(mesh, pf.SquirmerBC(), 0.05, "color", tol=pf.Tolerances(rtol_pres=1e-12))
sim.step(20)
sim.ctx.sync()
t = time.perf_counter()
st = sim.step(steps)
sim.ctx.sync()
el = time.perf_counter() - t
print(f"mesh_fine N={mesh.N}: {steps} steps in {el * 1e3:.2f} ms = {steps / el:.0f} steps/s "
      f"({el / steps * 1e6:.1f} us/step); path {sim.ctx.path_info()}")
sim.close()
