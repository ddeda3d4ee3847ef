"""Build libpucfem.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = ["csrc/pucfem_api.hip", "csrc/pucfem_host.cpp"]
DEPS = SRC + ["csrc/pucfem_host.hpp", "csrc/pucfem_kernels.hpp", "csrc/pucfem_kernels_impl.hpp",
              "csrc/pucfem_comm.hpp", "csrc/pucfem_lattice.hpp"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def build(force=False, verbose=False):
    out = os.path.join(HERE, "libpucfem.so")
    deps = [os.path.join(HERE, d) for d in DEPS] + [os.path.join(ROOT, "include", "pucfem.h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    cmd = [hipcc(), "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared", "-ffp-contract=off",
           "-Wall", "-Wno-unused-function", f"-I{os.path.join(ROOT, 'include')}", "-o", out + ".tmp"]
    cmd += [os.path.join(HERE, s) for s in SRC] + ["-lrccl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
