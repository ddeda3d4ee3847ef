"""The bench's mesh_fine leg (bench.secondary_fine) alone: GPU steps/s and the ratio to the on-host port.
  python tools/fine_leg.py [STEPS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from conftest import load_pkg  # noqa: E402

import bench  # noqa: E402

r = bench.secondary_fine(load_pkg(), int(sys.argv[1]) if len(sys.argv) > 1 else 2000)
print(os.environ.get("PUCFEM_GRAPH_STEPS", "default"), round(r["gpu_steps_per_s"]), round(r["ratio_vs_oracle"], 1))
