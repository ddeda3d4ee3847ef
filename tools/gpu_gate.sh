#!/bin/bash
# Round 6: the K-step small-mesh graph (bit identity, mesh_fine rate) and the dye tail's release point
# (PUCFEM_DYE_GATE 0 / 1 / 2) and the gated gradient projection (PUCFEM_GP_GATE): bit identity, then alternating
# driver-command benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-gate}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_long.py \
  -k "graph_of_k" > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -3 "$OUT/pytest.out"
for g in 1 8; do
  PUCFEM_GRAPH_STEPS=$g timeout -k 10 200 python - <<'PY' || exit 1
import os, sys, time
sys.path.insert(0, "tests")
from conftest import load_pkg
pf = load_pkg()
mesh = pf.load_mesh("fine")
sim = pf.StokesSimulation(mesh, pf.SquirmerBC(), 0.05, "color", tol=pf.Tolerances(rtol_pres=1e-12))
sim.step(20); sim.ctx.sync()
for rep in range(3):
    t = time.perf_counter(); sim.step(2000); sim.ctx.sync()
    print("graph steps", os.environ["PUCFEM_GRAPH_STEPS"], "mesh_fine", 2000 / (time.perf_counter() - t), "steps/s")
sim.close()
PY
done
for e in "PUCFEM_DYE_GATE=0" "PUCFEM_DYE_GATE=1" "PUCFEM_GP_GATE=0"; do
  echo "$e"; env $e timeout -k 10 300 python tools/bitcmp.py 7 30 || exit 1
done
for e in "PUCFEM_GP_GATE=1" "PUCFEM_GP_GATE=0"; do
  echo "$e"; env $e timeout -k 10 300 python tools/bitcmp.py 5 60 || exit 1
done
tools/gpu_env_ab.sh "$TAG" "" "PUCFEM_GP_GATE=0" "PUCFEM_DYE_GATE=1" "PUCFEM_DYE_GATE=2" "" "PUCFEM_GP_GATE=0" \
  "PUCFEM_DYE_GATE=1" "PUCFEM_DYE_GATE=1 PUCFEM_SL_BLOCKS=2048"
