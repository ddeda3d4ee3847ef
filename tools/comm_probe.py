"""Per-rank multi-GPU data flow of the StokesColor step on W LocalComm ranks (one GPU, one process):
the wide dye halo each rank receives vs a full all-gather, after each of S steps.
  python tools/comm_probe.py LEVEL W STEPS"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg  # noqa: E402

pf = load_pkg()
level, world, steps = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (5, 8, 6)))
mesh = pf.load_mesh("fine", refine=level)
uid = b"PUCFEM-LOCALCOMM" + os.urandom(112)
rows = [[None] * steps for _ in range(world)]
errs = []


def worker(r):
    try:
        sim = pf.StokesSimulation(mesh, pf.SquirmerBC(), 0.05, "color", 0, pf.Tolerances.production(),
                                  dist=(r, world, uid))
        for k in range(steps):
            sim.step(1)
            rows[r][k] = sim.ctx.comm_info()
        sim.close()
    except Exception as e:  # pragma: no cover
        errs.append((r, repr(e)))


th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
for t in th:
    t.start()
for t in th:
    t.join()
assert not errs, errs
print(f"L{level} N={mesh.N} W={world}")
for k in range(steps):
    h = [rows[r][k]["dye_halo_values"] for r in range(world)]
    a = [rows[r][k]["allgather_values"] for r in range(world)]
    print(f"step {k}: dye halo values per rank {h} (max {max(h) * 8 / 1e6:.2f} MB) vs all-gather "
          f"{max(a) * 8 / 1e6:.2f} MB")
