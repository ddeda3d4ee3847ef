"""Hash of the fields after K production steps (compare two builds bit for bit: run once per PUCFEM_LIB_VARIANT).
  python tools/bitcmp.py LEVEL STEPS"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg  # noqa: E402

pf = load_pkg()
level, steps = int(sys.argv[1]), int(sys.argv[2])
sim = pf.StokesSimulation(pf.load_mesh("fine", refine=level), pf.SquirmerBC(), 0.05, "color", 0, pf.Tolerances.production())
its = [(s.it_visc, s.it_p, s.it_p2) for k in (1, 4, steps - 5) for s in sim.step(k)]
h = hashlib.sha256()
for a in (sim.u, sim.c):
    h.update(a.tobytes())
print(os.environ.get("PUCFEM_LIB_VARIANT", "default"), f"L{level} {steps} steps", h.hexdigest()[:24], its[-3:])
sim.close()
