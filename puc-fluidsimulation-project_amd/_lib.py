"""ctypes binding of libpucfem.so (include/pucfem.h).

The library is built in-tree (``python -c "import __graft_entry__ as g; g.build()"``) and loaded
from this package directory.  There is no fallback: if the shared object is missing or a call
fails, a ``PucfemError`` is raised.
"""
from __future__ import annotations

import ctypes as ct
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBNAME = "libpucfem.so"

# enums (pucfem.h)
STOKES_COLOR, STOKES_FOOD, HEAT, POISSON = 0, 1, 2, 3
F_U, F_USTAR, F_P, F_P2, F_DIV_STAR, F_DIV_U, F_FINAL_DIV, F_C, F_SCALAR, F_TRACERS, F_STATUS = range(11)
OP_K, OP_VISC, OP_PRES, OP_GX, OP_GY, OP_DIV, OP_GRAD, OP_LIT, OP_MCONS, OP_MLUMP, OP_ASUM = range(11)
HOST_ONLY = -1
ERRORS = {-1: "EINVAL", -2: "EHIP", -3: "ENOCONV", -4: "ESTATE", -5: "ENCCL", -6: "ENOMEM", -7: "ENODEV"}


class PucfemError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"pucfem {ERRORS.get(code, code)}: {msg}")
        self.code = code


class Params(ct.Structure):
    _fields_ = [
        ("scheme", ct.c_int32), ("nstrips", ct.c_int32), ("dt", ct.c_double), ("nu", ct.c_double),
        ("rtol_visc", ct.c_double), ("rtol_pres", ct.c_double), ("rtol_lin", ct.c_double),
        ("maxit_visc", ct.c_int32), ("maxit_pres", ct.c_int32), ("maxit_lin", ct.c_int32),
        ("warm_start", ct.c_int32), ("sl_k", ct.c_int32), ("capture_radius", ct.c_double),
        ("center_x", ct.c_double), ("center_y", ct.c_double), ("precond", ct.c_int32),
        ("mg_degree", ct.c_int32), ("mg_ratio", ct.c_double), ("mg_post", ct.c_int32),
        ("mg_single", ct.c_int32), ("mg_rep_nodes", ct.c_int64), ("mg_f32_vals", ct.c_int32),
        ("idx32", ct.c_int32), ("proj_k", ct.c_int32), ("proj_k_visc", ct.c_int32), ("mg_kind", ct.c_int32),
        ("solver_path", ct.c_int32), ("assembled", ct.c_int32), ("dye_scheme", ct.c_int32),
        ("dye_diffusivity", ct.c_double), ("assembly", ct.c_int32), ("proj_shared", ct.c_int32),
    ]


class StepStats(ct.Structure):
    _fields_ = [
        ("max_div_star", ct.c_double), ("max_final_div", ct.c_double), ("mix_I", ct.c_double),
        ("mix_mu", ct.c_double), ("mix_var", ct.c_double), ("eaten", ct.c_int64), ("it_visc", ct.c_int32),
        ("it_p", ct.c_int32), ("it_p2", ct.c_int32), ("sl_notfound", ct.c_int32),
    ]


_P = ct.c_void_p
_D = ct.POINTER(ct.c_double)
_I32 = ct.POINTER(ct.c_int32)
_I64 = ct.POINTER(ct.c_int64)
_F = ct.POINTER(ct.c_float)
_U8 = ct.POINTER(ct.c_uint8)

SIGNATURES = {
    "pucfem_abi_version": ([], ct.c_int),
    "pucfem_last_error": ([_P], ct.c_char_p),
    "pucfem_device_count": ([_I32], ct.c_int),
    "pucfem_ctx_create": ([ct.c_int32, ct.POINTER(_P)], ct.c_int),
    "pucfem_rccl_unique_id": ([_U8], ct.c_int),
    "pucfem_ctx_create_dist": ([ct.c_int32, ct.c_int32, ct.c_int32, _U8, ct.POINTER(_P)], ct.c_int),
    "pucfem_ctx_destroy": ([_P], ct.c_int),
    "pucfem_mesh_upload": ([_P, ct.c_int64, _D, _I32, ct.c_int64, _I32, ct.c_int32], ct.c_int),
    "pucfem_set_pairs": ([_P, ct.c_int32, ct.c_int64, _I64], ct.c_int),
    "pucfem_set_dirichlet": ([_P, ct.c_int64, _I32, _D, ct.c_int32], ct.c_int),
    "pucfem_set_source": ([_P, ct.c_int64, _F], ct.c_int),
    "pucfem_set_hierarchy": ([_P, ct.c_int64, _D, _I32, ct.c_int64, _I32, ct.c_int32], ct.c_int),
    "pucfem_build_operators": ([_P, ct.POINTER(Params)], ct.c_int),
    "pucfem_set_field": ([_P, ct.c_int32, _D, ct.c_int64], ct.c_int),
    "pucfem_get_field": ([_P, ct.c_int32, _D, ct.c_int64], ct.c_int),
    "pucfem_step": ([_P, ct.c_int32, ct.POINTER(StepStats)], ct.c_int),
    "pucfem_apply": ([_P, ct.c_int32, _D, _D], ct.c_int),
    "pucfem_solve": ([_P, ct.c_int32, _D, _D, ct.c_double, ct.c_int32, _I32], ct.c_int),
    "pucfem_sl_advect": ([_P, _D, _D, ct.c_double, _D, _I32], ct.c_int),
    "pucfem_apply_bc": ([_P, ct.c_int32, _D], ct.c_int),
    "pucfem_dye_step": ([_P, _D, _D, _D, _I32], ct.c_int),
    "pucfem_comm_info": ([_P, ct.POINTER(ct.c_int64)], ct.c_int),
    "pucfem_visc_interval": ([_P, ct.POINTER(ct.c_double)], ct.c_int),
    "pucfem_mg_lmax": ([_P, ct.c_int32, _D], ct.c_int),
    "pucfem_proj_info": ([_P, _D], ct.c_int),
    "pucfem_tracer_step": ([_P, _D, ct.c_double, ct.c_int32], ct.c_int),
    "pucfem_mixing_index": ([_P, _D, _D], ct.c_int),
    "pucfem_mixing_index_w": ([_P, _D, _D, _D], ct.c_int),
    "pucfem_comm_selftest": ([_P, _D], ct.c_int),
    "pucfem_cgcg_coef_probe": ([_P, _D, ct.c_double, _D, ct.c_double, ct.c_int32, ct.c_int32, ct.c_double, _I32, _D],
                               ct.c_int),
    "pucfem_timing_enable": ([_P, ct.c_int32], ct.c_int),
    "pucfem_timing_get": ([_P, ct.c_int32, _D, _I64, _D], ct.c_int),
    "pucfem_counters": ([_P, _I64, _D], ct.c_int),
    "pucfem_class_counters": ([_P, ct.c_int32, _I64, _D], ct.c_int),
    "pucfem_comm_counters": ([_P, _I64], ct.c_int),
    "pucfem_sync": ([_P], ct.c_int),
    "pucfem_bench_dir": ([_P, ct.c_int32, ct.c_int32, ct.c_int32, _D], ct.c_int),
    "pucfem_bench_kernel": ([_P, ct.c_int32, ct.c_int32, _D, _D, _D], ct.c_int),
    "pucfem_info": ([_P, _I64], ct.c_int),
    "pucfem_path_info": ([_P, _I64], ct.c_int),
    "pucfem_refine": ([ct.c_int64, _D, _I32, ct.c_int64, _I32, ct.c_int32, _I64, _I64, _D, _I32, _I32], ct.c_int),
    "pucfem_host_get_csr": ([_P, ct.c_int32, _I64, _I64, _I64, _I64, _D], ct.c_int),
    "pucfem_host_lattice_apply": ([_P, ct.c_int32, ct.c_int32, _D, _D], ct.c_int),
    "pucfem_host_partition": ([_P, ct.c_int32, ct.c_int32, _I64, _I64, _I64, _I64, _I32, _I64, _I64, _I32], ct.c_int),
}

_lib = None


def lib_path():
    # PUCFEM_LIB_VARIANT=v loads libpucfem.v.so from the same directory (A/B builds of the measurement
    # tools; the default is the library __graft_entry__.build() makes)
    v = os.environ.get("PUCFEM_LIB_VARIANT")
    if v:
        if os.path.basename(v) != v:
            raise PucfemError(-1, "PUCFEM_LIB_VARIANT is a bare variant name")
        return os.path.join(HERE, f"libpucfem.{v}.so")
    return os.path.join(HERE, LIBNAME)


def lib():
    """Load libpucfem.so from the package directory (raises if it has not been built)."""
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise PucfemError(-7, f"{path} not built: run __graft_entry__.build()")
        L = ct.CDLL(path)
        for name, (args, res) in SIGNATURES.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != 0:
        msg = lib().pucfem_last_error(ctx)
        raise PucfemError(rc, msg.decode() if msg else "")


def dptr(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_D)


def iptr(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_I32)


def lptr(a):
    assert a.dtype == np.int64 and a.flags.c_contiguous
    return a.ctypes.data_as(_I64)


def fptr(a):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_F)


def device_count():
    n = ct.c_int32(0)
    rc = lib().pucfem_device_count(ct.byref(n))
    return n.value if rc == 0 else 0
