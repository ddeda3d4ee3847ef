"""The C ABI (include/*.h) against the built library and the ctypes binding -- no device needed.

Every function the public header declares must be exported by libpucfem.so and bound (argument and
result types) in _lib.SIGNATURES; the params / stats structs must have the header's field order.
"""
import ctypes as ct
import glob
import os
import re

import pytest

from conftest import ROOT, load_pkg

pf = load_pkg()
from importlib import import_module  # noqa: E402

L = import_module("puc-fluidsimulation-project_amd._lib")

DECL = re.compile(r"^\s*(?:const\s+)?\w+\s*\*?\s*(pucfem_\w+)\s*\(", re.M)


def header_functions():
    names = []
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names += DECL.findall(text)
    return sorted(set(names))


def test_header_declares_the_abi():
    names = header_functions()
    assert "pucfem_step" in names and "pucfem_ctx_create" in names and "pucfem_path_info" in names
    assert len(names) >= 30


@pytest.mark.parametrize("name", header_functions())
def test_symbol_exported_and_bound(name):
    lib = L.lib()
    assert hasattr(lib, name), f"{name} declared in include/pucfem.h but not exported by libpucfem.so"
    assert name in L.SIGNATURES, f"{name} has no ctypes signature in _lib.SIGNATURES"
    # the binding's declared arity is what the C declaration takes
    hdr = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "pucfem.h")).read(), flags=re.S)
    m = re.search(rf"{name}\s*\(([^)]*)\)", hdr)
    params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
    assert len(params) == len(L.SIGNATURES[name][0]), name


def test_params_struct_matches_header():
    hdr = open(os.path.join(ROOT, "include", "pucfem.h")).read()
    body = hdr[hdr.index("typedef struct pucfem_params"):hdr.index("} pucfem_params;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"(int32_t|int64_t|double)\s+([\w\s,]+);", body)
    names = [n.strip() for _, group in fields for n in group.split(",")]
    assert names == [f[0] for f in L.Params._fields_]
    ctypes_of = {"int32_t": ct.c_int32, "int64_t": ct.c_int64, "double": ct.c_double}
    types = [ctypes_of[t] for t, group in fields for _ in group.split(",")]
    assert types == [f[1] for f in L.Params._fields_]


def test_abi_version_and_host_only_context():
    lib = L.lib()
    assert lib.pucfem_abi_version() == 1
    p = ct.c_void_p()
    L.check(lib.pucfem_ctx_create(L.HOST_ONLY, ct.byref(p)))
    # a compute call on a host-only context fails loudly (no CPU fallback)
    rc = lib.pucfem_sync(p)
    assert rc == 0
    o = (ct.c_int64 * 8)()
    assert lib.pucfem_path_info(p, o) == -4  # ESTATE: not built
    assert b"build" in lib.pucfem_last_error(p)
    L.check(lib.pucfem_ctx_destroy(p))
