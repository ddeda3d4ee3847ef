"""Hash of the mesh_fine fields and step records after K steps of the small-mesh (graph) path (compare builds or
knobs bit for bit: run once per PUCFEM_LIB_VARIANT / setting).
  python tools/bitcmp_fine.py STEPS"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg  # noqa: E402

pf = load_pkg()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
sim = pf.StokesSimulation(pf.load_mesh("fine"), pf.SquirmerBC(), 0.05, "color", 0, pf.Tolerances(rtol_pres=1e-12))
st = sim.step(steps)
h = hashlib.sha256()
for a in (sim.u, sim.c):
    h.update(a.tobytes())
h.update(repr([(s.max_div_star, s.max_final_div, s.mix_var) for s in st]).encode())
print(os.environ.get("PUCFEM_LIB_VARIANT", "default"), f"mesh_fine {steps} steps", h.hexdigest()[:24])
sim.close()
