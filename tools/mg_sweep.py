#!/usr/bin/env python3
"""Multigrid smoother parameter sweep: pressure-solve iterations and time (one GPU)."""
import importlib, json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pf = importlib.import_module("puc-fluidsimulation-project_amd")
L = importlib.import_module("puc-fluidsimulation-project_amd._lib")
level = int(sys.argv[1]) if len(sys.argv) > 1 else 5
mesh = pf.load_mesh("fine", refine=level)
rng = np.random.default_rng(0)
b = None
for pre, post, ratio in [(2, 2, 10), (1, 1, 10), (1, 2, 10), (2, 1, 10), (3, 3, 10), (2, 2, 4), (2, 2, 30), (1, 1, 4), (3, 2, 10)]:
    tol = pf.Tolerances(precond="mg", mg_degree=pre, mg_post=post, mg_ratio=ratio)
    sim = pf.StokesSimulation(mesh, pf.SquirmerBC(), 0.05, "color", tol=tol)
    if b is None:
        u = rng.standard_normal((mesh.N, 2))
        b = -20.0 * sim.ctx.apply(L.OP_DIV, u, (mesh.N,))
    sim.ctx.solve(L.OP_PRES, b, rtol=1e-8)
    sim.ctx.sync()
    t = time.perf_counter()
    _, it = sim.ctx.solve(L.OP_PRES, b, rtol=1e-8)
    dt = time.perf_counter() - t
    print(json.dumps({"level": level, "pre": pre, "post": post, "ratio": ratio, "iters": it, "ms": 1e3 * dt}), flush=True)
    sim.close()
