"""lbm_amd -- Python bindings of liblbm.so (the HIP D3Q19 hot path) and liblbm_host.so
(the per-case host ingest/output), used by tests/, bench.py and __graft_entry__.py.

The product is the C ABI declared in include/lbm.h and include/lbm_host.h; this module
only marshals numpy arrays through ctypes.  There is no CPU fallback: every solver
call goes to liblbm.so, and a missing library or device raises.

torch is imported before liblbm.so is loaded so that both share one HIP runtime (the
wheel bundles its own libamdhip64.so.7/librccl.so.1; liblbm.so's DT_NEEDED sonames
then resolve to those copies instead of loading a second runtime).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

try:  # shared HIP runtime (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                      # lattice-boltzmann-method-gpu_amd/
LIB = os.path.join(ROOT, "lib")
LIBLBM = os.environ.get("LBM_LIBRARY") or os.path.join(LIB, "liblbm.so")  # override: A/B builds
LIBHOST = os.path.join(LIB, "liblbm_host.so")

LBM_CASE_LDC, LBM_CASE_POISEUILLE, LBM_CASE_MASK, LBM_CASE_GENERIC = 0, 1, 2, 3
LBM_FACE_PX, LBM_FACE_NX, LBM_FACE_PY, LBM_FACE_NY, LBM_FACE_PZ, LBM_FACE_NZ = range(6)
LBM_BC_VELOCITY, LBM_BC_VELOCITY_RHO, LBM_BC_PRESSURE = 0, 1, 2
LBM_INIT_LDC_WI, LBM_INIT_EXPANDED = 0, 1
LBM_SUM_FP64, LBM_SUM_CUB_TREE = 0, 1  # lbm_set_residual_order
# lbm_tune knobs (include/lbm.h lbm_tune_knob)
(TUNE_ROW_AXIS, TUNE_CELLS_PER_LANE, TUNE_EXACT_DIV, TUNE_FUSED_RESIDUAL, TUNE_BUFFER_ALLOC,
 TUNE_SYNC_TIMEOUT_S, TUNE_GRID_STRIDE, TUNE_INJECT_RCCL_FAULT, TUNE_GROUPS, TUNE_GROUP_SEGMENT, TUNE_COMPACT,
 TUNE_BOX, TUNE_NEE_FIX, TUNE_XCD_RUN, TUNE_NEE_ORDER) = range(15)

# reference per-case constants
LDC_TAU, LDC_C_U, LDC_CH = 0.55, 2.4705, 0.0000655737                   # ldc.cu:49,55
POIS_TAU, POIS_C_U, POIS_UMAX_KERNEL = 0.58, 1.5441, 0.09714700668       # Poiseulle.cu:39,590
BIF_TAU, BIF_C_U, BIF_CH = 0.55, 0.24159041, 0.000248925                 # bifurcation.cu:20,434
BIF_SHAPE = (32, 83, 64)                                                 # (nz, ny, nx)


def lid_u() -> float:
    """u_max = 0.15f / C_U of ldc.cu:52, rounded in fp32 like the reference."""
    return float(np.float32(0.15) / np.float32(LDC_C_U))


class LbmError(RuntimeError):
    pass


class lbm_bc_code(C.Structure):
    _fields_ = [
        ("code", C.c_int), ("face", C.c_int), ("kind", C.c_int),
        ("rho", C.c_float), ("u", C.c_float * 3),
        ("u_normal_table", C.POINTER(C.c_float)),
    ]


class lbm_desc(C.Structure):
    _fields_ = [
        ("nx", C.c_int), ("ny", C.c_int), ("nz", C.c_int),
        ("tau", C.c_float),
        ("case_kind", C.c_int),
        ("geo", C.POINTER(C.c_int8)),
        ("halo_planes", C.c_int),
        ("lid_u", C.c_float),
        ("bc_inlet_uy", C.POINTER(C.c_float)),
        ("bc_outlet_uy", C.POINTER(C.c_float)),
        ("device", C.c_int),
        ("z_offset", C.c_int),
        ("nz_global", C.c_int),
        ("x_align", C.c_int),
        ("bc_codes", C.POINTER(lbm_bc_code)),
        ("n_bc_codes", C.c_int),
        ("mask", C.POINTER(C.c_uint8)),
        ("row_axis", C.c_int),
    ]


# every symbol include/lbm.h and include/lbm_host.h declare (checked by the CPU tests)
LBM_SYMBOLS = [
    "lbm_version", "lbm_last_error", "lbm_tune", "lbm_get_nonfinite", "lbm_create", "lbm_destroy", "lbm_init_equilibrium", "lbm_init_ldc",
    "lbm_init_case", "lbm_set_f", "lbm_field_digest", "lbm_set_convergence", "lbm_set_residual_order", "lbm_step", "lbm_sync", "lbm_get_state", "lbm_get_macros", "lbm_get_f",
    "lbm_get_geo", "lbm_get_counts", "lbm_profile", "lbm_stats", "lbm_kernel_times", "lbm_get_boundary_cells", "lbm_get_storage", "lbm_get_numerics",
    "lbm_get_nee_path", "lbm_get_setup_cost",
    "lbm_get_layout", "lbm_get_launch_shape", "lbm_buffer_placement", "lbm_checkpoint_save", "lbm_checkpoint_load",
    "lbm_rccl_unique_id", "lbm_attach_rccl", "lbm_comm_info", "lbm_debug_fail_next_wait", "lbm_debug_poison_walls",
    "lbm_group_step", "lbm_probe_stream", "lbm_probe_stream_shapes",
]
HOST_SYMBOLS = [
    "lbmh_geo_ldc", "lbmh_geo_poiseuille", "lbmh_geo_mask", "lbmh_read_geo_txt", "lbmh_read_bc_txt",
    "lbmh_index_transform", "lbmh_poiseuille_profile", "lbmh_initial_fields", "lbmh_write_vtk", "lbmh_calc_res",
    "lbmh_read_geo_txt_zxy", "lbmh_geo_ends", "lbmh_coronary_ends", "lbmh_write_vtk_coronary", "lbmh_calc_res_fluid",
]


class lbmh_end(C.Structure):
    """include/lbm_host.h lbmh_end: one open end of a vessel mask (coronary.cu:75-143)."""
    _fields_ = [(n, C.c_int) for n in ("axis", "plane", "lo0", "hi0", "lo1", "hi1", "passes")]

_lbm = None
_host = None

i8p = C.POINTER(C.c_int8)
i32p = C.POINTER(C.c_int32)
f32p = C.POINTER(C.c_float)
f64p = C.POINTER(C.c_double)
i64p = C.POINTER(C.c_int64)
ip = C.POINTER(C.c_int)
P = C.c_void_p


def _ptr(a: np.ndarray | None, ct):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ct))


def host_lib() -> C.CDLL:
    global _host
    if _host is None:
        if not os.path.exists(LIBHOST):
            raise LbmError(f"{LIBHOST} missing: run `make -C {ROOT}` or __graft_entry__.build()")
        L = C.CDLL(LIBHOST)
        sig = {
            "lbmh_geo_ldc": (None, [C.c_int, C.c_int, C.c_int, i8p]),
            "lbmh_geo_poiseuille": (None, [C.c_int, C.c_int, C.c_int, i8p]),
            "lbmh_geo_mask": (None, [C.c_int, C.c_int, C.c_int, i32p, i8p]),
            "lbmh_read_geo_txt": (C.c_long, [C.c_char_p, C.c_int, C.c_int, C.c_int, i32p]),
            "lbmh_read_bc_txt": (C.c_long, [C.c_char_p, C.c_int, C.c_int, C.c_int, i8p, C.c_int, f32p, f32p]),
            "lbmh_index_transform": (C.c_int64, [C.c_int, C.c_int, C.c_int, i8p, i32p]),
            "lbmh_poiseuille_profile": (None, [C.c_int, C.c_int, C.c_float, f32p]),
            "lbmh_initial_fields": (None, [C.c_int, C.c_int, C.c_int, C.c_int, i8p, f32p, f32p, f32p, f32p, f32p, f32p]),
            "lbmh_write_vtk": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, i8p, f32p, f32p, f32p,
                                         C.c_float, C.c_float]),
            "lbmh_calc_res": (C.c_longdouble, [C.c_int, C.c_int, C.c_int, i8p, f32p, f32p, f32p]),
            "lbmh_read_geo_txt_zxy": (C.c_long, [C.c_char_p, C.c_int, C.c_int, C.c_int, i32p]),
            "lbmh_calc_res_fluid": (C.c_longdouble, [C.c_int, C.c_int, C.c_int, i8p, f32p, f32p, f32p]),
            "lbmh_geo_ends": (C.c_int, [C.c_int, C.c_int, C.c_int, i32p, C.c_int, C.POINTER(lbmh_end), i8p]),
            "lbmh_coronary_ends": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(lbmh_end)]),
            "lbmh_write_vtk_coronary": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, i8p, f32p, f32p, f32p, f32p,
                                                  C.c_float, C.c_float, C.c_float]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _host = L
    return _host


def lbm_lib() -> C.CDLL:
    global _lbm
    if _lbm is None:
        if not os.path.exists(LIBLBM):
            raise LbmError(f"{LIBLBM} missing: run `make -C {ROOT}` or __graft_entry__.build()")
        L = C.CDLL(LIBLBM)
        sig = {
            "lbm_version": (C.c_char_p, []),
            "lbm_last_error": (C.c_char_p, [P]),
            "lbm_tune": (C.c_int, [C.c_int, C.c_int]),
            "lbm_get_nonfinite": (C.c_int, [P, ip]),
            "lbm_create": (C.c_int, [C.POINTER(lbm_desc), C.POINTER(P)]),
            "lbm_destroy": (None, [P]),
            "lbm_init_equilibrium": (C.c_int, [P, C.c_int, f32p, f32p, f32p, f32p]),
            "lbm_init_ldc": (C.c_int, [P]),
            "lbm_init_case": (C.c_int, [P]),
            "lbm_set_f": (C.c_int, [P, f32p]),
            "lbm_set_convergence": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_float]),
            "lbm_set_residual_order": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int]),
            "lbm_step": (C.c_int, [P, C.c_int, f32p, ip]),
            "lbm_sync": (C.c_int, [P]),
            "lbm_get_state": (C.c_int, [P, ip, ip, ip, f32p, f64p]),
            "lbm_get_macros": (C.c_int, [P, f32p, f32p, f32p, f32p]),
            "lbm_get_f": (C.c_int, [P, f32p]),
            "lbm_field_digest": (C.c_int, [P, C.POINTER(C.c_uint64)]),
            "lbm_get_geo": (C.c_int, [P, C.POINTER(C.c_int8)]),
            "lbm_get_counts": (C.c_int, [P, i64p, i64p, f64p]),
            "lbm_profile": (C.c_int, [P, C.c_int]),
            "lbm_stats": (C.c_int, [P, f64p, i64p, f64p]),
            "lbm_kernel_times": (C.c_int, [P, C.c_int, f64p, i64p]),
            "lbm_get_boundary_cells": (C.c_int, [P, i64p]),
            "lbm_get_storage": (C.c_int, [P, ip, i64p, i64p]),
            "lbm_get_nee_path": (C.c_int, [P, ip, ip]),
            "lbm_get_setup_cost": (C.c_int, [P, f64p, i64p, i64p]),
            "lbm_checkpoint_save": (C.c_int, [P, C.c_char_p]),
            "lbm_checkpoint_load": (C.c_int, [P, C.c_char_p]),
            "lbm_get_numerics": (C.c_int, [P, ip, i64p]),
            "lbm_get_layout": (C.c_int, [P, ip, ip, ip, i64p]),
            "lbm_get_launch_shape": (C.c_int, [P, ip, ip, ip, C.POINTER(C.c_double)]),
            "lbm_buffer_placement": (C.c_int, [P, f64p, C.c_int, ip, ip]),
            "lbm_rccl_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
            "lbm_attach_rccl": (C.c_int, [P, C.POINTER(C.c_uint8), C.c_int, C.c_int]),
            "lbm_comm_info": (C.c_int, [P, ip, ip]),
            "lbm_debug_fail_next_wait": (C.c_int, [P]),
            "lbm_debug_poison_walls": (C.c_int, [P]),
            "lbm_group_step": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, f32p]),
            "lbm_probe_stream": (C.c_int, [C.c_int, C.c_int64, C.c_int, f64p]),
            "lbm_probe_stream_shapes": (C.c_int, [C.c_int, C.c_int64, C.c_int, f64p, C.c_int, ip]),
        }
        for name, (res, args) in sig.items():
            # an A/B build named by LBM_LIBRARY may predate an entry point; the product may not
            if os.environ.get("LBM_LIBRARY") and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lbm = L
    return _lbm


def kernel_fingerprint() -> str:
    """16 hex digits identifying the code of liblbm's kernels and launch logic: sha256 of
    csrc/lbm_kernels.hip, lbm_kernels.hpp, lbm_d3q19.hpp and lbm_ctx.hip with // comments and
    whitespace removed.  Profiles record it (tools/pmc_*.py) so that bench.py reports measured
    HBM traffic only next to the kernels it was measured on."""
    import hashlib
    import re
    h = hashlib.sha256()
    for name in ("lbm_kernels.hip", "lbm_kernels.hpp", "lbm_d3q19.hpp", "lbm_ctx.hip"):
        text = open(os.path.join(ROOT, "csrc", name)).read()
        text = re.sub(r"//[^\n]*", "", text)
        h.update(re.sub(r"\s+", "", text).encode())
    return h.hexdigest()[:16]


def version() -> str:
    return lbm_lib().lbm_version().decode()


def tune(knob: int, value: int) -> int:
    """Set a process-wide lbm_tune knob (read at context creation); returns the old value."""
    prev = lbm_lib().lbm_tune(knob, value)
    if prev < 0:
        raise LbmError(f"lbm_tune({knob}, {value}): {lbm_lib().lbm_last_error(None).decode()}")
    return prev


class tuned:
    """Context manager: `with tuned(TUNE_ROW_AXIS, 1): ...` restores the old value on exit."""

    def __init__(self, knob: int, value: int):
        self.knob, self.value = knob, value

    def __enter__(self):
        self.prev = tune(self.knob, self.value)
        return self

    def __exit__(self, *exc):
        tune(self.knob, self.prev)
        return False


# ---------------------------------------------------------------------------------------
# host ingest (liblbm_host.so)
# ---------------------------------------------------------------------------------------

def geo_ldc(nx: int, ny: int, nz: int) -> np.ndarray:
    g = np.zeros((nz, ny, nx), np.int8)
    host_lib().lbmh_geo_ldc(nx, ny, nz, _ptr(g, C.c_int8))
    return g


def geo_poiseuille(nx: int, ny: int, nz: int) -> np.ndarray:
    g = np.zeros((nz, ny, nx), np.int8)
    host_lib().lbmh_geo_poiseuille(nx, ny, nz, _ptr(g, C.c_int8))
    return g


def read_geo_txt(path: str, shape=BIF_SHAPE) -> np.ndarray:
    nz, ny, nx = shape
    raw = np.zeros(shape, np.int32)
    n = host_lib().lbmh_read_geo_txt(path.encode(), nx, ny, nz, _ptr(raw, C.c_int32))
    if n != raw.size:
        raise LbmError(f"{path}: read {n} of {raw.size} mask values")
    return raw


def geo_mask(raw: np.ndarray) -> np.ndarray:
    raw = np.ascontiguousarray(raw, np.int32)
    nz, ny, nx = raw.shape
    g = np.zeros(raw.shape, np.int8)
    host_lib().lbmh_geo_mask(nx, ny, nz, _ptr(raw, C.c_int32), _ptr(g, C.c_int8))
    return g


def read_geo_txt_zxy(path: str, shape) -> np.ndarray:
    """coronary.cu:45-56: geo.txt in z, x, y loop order; returns the raster [nz][ny][nx]."""
    nz, ny, nx = shape
    raw = np.zeros(shape, np.int32)
    n = host_lib().lbmh_read_geo_txt_zxy(path.encode(), nx, ny, nz, _ptr(raw, C.c_int32))
    if n != raw.size:
        raise LbmError(f"{path}: read {n} of {raw.size} mask values")
    return raw


def coronary_ends(shape):
    """The reference's five vessel ends for a box of this shape (lbmh_coronary_ends) as tuples
    (axis, plane, lo0, hi0, lo1, hi1, passes)."""
    nz, ny, nx = shape
    arr = (lbmh_end * 5)()
    if host_lib().lbmh_coronary_ends(nx, ny, nz, arr) != 5:
        raise LbmError(f"box {nx}x{ny}x{nz} cannot hold coronary.cu's end planes (needs >= 274x201x206)")
    return [tuple(getattr(e, f) for f, _ in lbmh_end._fields_) for e in arr]


def geo_ends(raw: np.ndarray, ends) -> np.ndarray:
    """geo_pre of a vessel mask with open ends (lbmh_geo_ends, coronary.cu:31-275)."""
    raw = np.ascontiguousarray(raw, np.int32)
    nz, ny, nx = raw.shape
    arr = (lbmh_end * max(1, len(ends)))(*[lbmh_end(*e) for e in ends])
    g = np.zeros(raw.shape, np.int8)
    if host_lib().lbmh_geo_ends(nx, ny, nz, _ptr(raw, C.c_int32), len(ends), arr, _ptr(g, C.c_int8)) != 0:
        raise LbmError(f"lbmh_geo_ends: an end of {list(ends)} leaves the {nx}x{ny}x{nz} box's interior")
    return g


def write_vtk_coronary(path: str, geo: np.ndarray, rho, ux, uy, uz, C_U: float = 2.74909090909091,
                       CH: float = 6.1111e-05, C_rho: float = 1060.0) -> None:
    g = np.ascontiguousarray(geo, np.int8)
    nz, ny, nx = g.shape
    arrs = [np.ascontiguousarray(a, np.float32) for a in (rho, ux, uy, uz)]
    rc = host_lib().lbmh_write_vtk_coronary(path.encode(), nx, ny, nz, _ptr(g, C.c_int8),
                                            *[_ptr(a, C.c_float) for a in arrs], C_U, CH, C_rho)
    if rc != 0:
        raise LbmError(f"cannot write {path}")


def read_bc_txt(path: str, geo, inlet_block: int = 0):
    """geo: the codes (entries off code-2 / code-3 cells are zeroed), or a (nz, ny, nx) shape
    for the unmasked tables (the device-built mask path masks them itself)."""
    g = None if isinstance(geo, tuple) else np.ascontiguousarray(geo, np.int8)
    nz, ny, nx = geo if g is None else g.shape
    inl = np.zeros((nz, nx), np.float32)
    out = np.zeros((nz, nx), np.float32)
    n = host_lib().lbmh_read_bc_txt(path.encode(), nx, ny, nz, _ptr(g, C.c_int8),
                                    inlet_block, _ptr(inl, C.c_float), _ptr(out, C.c_float))
    if n < 0:
        raise LbmError(f"cannot read {path}")
    return int(n), inl, out


def index_transform(geo: np.ndarray):
    g = np.ascontiguousarray(geo, np.int8)
    nz, ny, nx = g.shape
    idx = np.zeros(g.shape, np.int32)
    n = host_lib().lbmh_index_transform(nx, ny, nz, _ptr(g, C.c_int8), _ptr(idx, C.c_int32))
    return int(n), idx


def poiseuille_profile(nx: int, nz: int, u_max: float = POIS_UMAX_KERNEL) -> np.ndarray:
    t = np.zeros((nz, nx), np.float32)
    host_lib().lbmh_poiseuille_profile(nx, nz, u_max, _ptr(t, C.c_float))
    return t


def x_align_for(geo: np.ndarray, case_kind: int) -> int:
    """lbm_desc.x_align the library would choose for this whole-lattice mask (give the same
    value to every slab of it): the most common first-fluid x of a row onto a 4-cell boundary."""
    fluid = 3 if case_kind == LBM_CASE_LDC else 4
    g = np.ascontiguousarray(geo, np.int8).reshape(-1, geo.shape[-1]) == fluid
    has = g.any(axis=1)
    first = np.argmax(g, axis=1)[has]
    hist = np.bincount(first & 3, minlength=4)
    return int(np.argmax(hist)) + 1


def initial_fields(case_kind: int, geo: np.ndarray, inlet_uy=None, outlet_uy=None):
    g = np.ascontiguousarray(geo, np.int8)
    nz, ny, nx = g.shape
    out = [np.zeros(g.shape, np.float32) for _ in range(4)]
    inl = None if inlet_uy is None else np.ascontiguousarray(inlet_uy, np.float32)
    outl = None if outlet_uy is None else np.ascontiguousarray(outlet_uy, np.float32)
    host_lib().lbmh_initial_fields(case_kind, nx, ny, nz, _ptr(g, C.c_int8), _ptr(inl, C.c_float),
                                   _ptr(outl, C.c_float), *[_ptr(a, C.c_float) for a in out])
    return tuple(out)


def write_vtk(path: str, case_kind: int, geo: np.ndarray, ux, uy, uz, C_U: float, CH: float) -> None:
    g = np.ascontiguousarray(geo, np.int8)
    nz, ny, nx = g.shape
    arrs = [np.ascontiguousarray(a, np.float32) for a in (ux, uy, uz)]
    rc = host_lib().lbmh_write_vtk(path.encode(), case_kind, nx, ny, nz, _ptr(g, C.c_int8),
                                   *[_ptr(a, C.c_float) for a in arrs], C_U, CH)
    if rc != 0:
        raise LbmError(f"cannot write {path}")


def calc_res(geo: np.ndarray, ux, uy, uz) -> float:
    g = np.ascontiguousarray(geo, np.int8)
    nz, ny, nx = g.shape
    arrs = [np.ascontiguousarray(a, np.float32) for a in (ux, uy, uz)]
    return float(host_lib().lbmh_calc_res(nx, ny, nz, _ptr(g, C.c_int8), *[_ptr(a, C.c_float) for a in arrs]))


# ---------------------------------------------------------------------------------------
# solver contexts (liblbm.so)
# ---------------------------------------------------------------------------------------

class Lattice:
    """One liblbm context: a lattice, or one z-slab of it, on one GPU."""

    def __init__(self, case_kind: int, shape, tau: float, geo: np.ndarray | None = None, *,
                 halo_planes: bool = False, lid_u_val: float | None = None, inlet_uy=None, outlet_uy=None,
                 device: int = 0, z_offset: int = 0, nz_global: int | None = None, x_align: int = 0,
                 bc_codes=None, mask: np.ndarray | None = None, row_axis: int = 0):
        """mask (LBM_CASE_MASK, geo None): raw geo.txt mask, uint8 [nz (+6 with halo_planes)][ny][nx];
        geo_pre runs on the device (lbm_desc.mask)."""
        nz, ny, nx = shape
        self.shape = (nz, ny, nx)
        self.case_kind = case_kind
        d = lbm_desc()
        d.nx, d.ny, d.nz = nx, ny, nz
        d.tau = tau
        d.case_kind = case_kind
        self._keep = []
        if geo is not None:
            g = np.ascontiguousarray(geo, np.int8)
            want = (nz + 2 if halo_planes else nz, ny, nx)
            if g.shape != want:
                raise LbmError(f"geo shape {g.shape} != {want}")
            self._keep.append(g)
            d.geo = _ptr(g, C.c_int8)
        if mask is not None:
            m = np.ascontiguousarray(mask, np.uint8)
            want = (nz + 6 if halo_planes else nz, ny, nx)
            if m.shape != want:
                raise LbmError(f"mask shape {m.shape} != {want}")
            self._keep.append(m)
            d.mask = _ptr(m, C.c_uint8)
        d.halo_planes = 1 if halo_planes else 0
        d.lid_u = lid_u() if lid_u_val is None else lid_u_val
        for name, tab in (("bc_inlet_uy", inlet_uy), ("bc_outlet_uy", outlet_uy)):
            if tab is not None:
                t = np.ascontiguousarray(tab, np.float32)
                self._keep.append(t)
                setattr(d, name, _ptr(t, C.c_float))
        d.device = device
        d.z_offset = z_offset
        d.nz_global = nz if nz_global is None else nz_global
        d.x_align = x_align
        d.row_axis = row_axis
        if bc_codes:
            arr = (lbm_bc_code * len(bc_codes))()
            for k, b in enumerate(bc_codes):
                arr[k].code, arr[k].face, arr[k].kind = b["code"], b["face"], b["kind"]
                arr[k].rho = b.get("rho", 1.0)
                for i, v in enumerate(b.get("u", (0.0, 0.0, 0.0))):
                    arr[k].u[i] = v
                if b.get("table") is not None:
                    t = np.ascontiguousarray(b["table"], np.float32)
                    self._keep.append(t)
                    arr[k].u_normal_table = _ptr(t, C.c_float)
            self._keep.append(arr)
            d.bc_codes = C.cast(arr, C.POINTER(lbm_bc_code))
            d.n_bc_codes = len(bc_codes)
        self.desc = d
        h = P()
        rc = lbm_lib().lbm_create(C.byref(d), C.byref(h))
        if rc != 0:
            raise LbmError(f"lbm_create: {lbm_lib().lbm_last_error(None).decode()}")
        self.h = h

    def _ck(self, rc: int, what: str):
        if rc != 0:
            raise LbmError(f"{what}: {lbm_lib().lbm_last_error(self.h).decode()}")

    def close(self):
        if getattr(self, "h", None):
            lbm_lib().lbm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def init_equilibrium(self, form: int, rho=None, ux=None, uy=None, uz=None):
        arrs = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (rho, ux, uy, uz)]
        self._ck(lbm_lib().lbm_init_equilibrium(self.h, form, *[_ptr(a, C.c_float) for a in arrs]),
                 "lbm_init_equilibrium")

    def init_ldc(self):
        self._ck(lbm_lib().lbm_init_ldc(self.h), "lbm_init_ldc")

    def init_case(self):
        """The case's initialize() on the device (LDC, MASK)."""
        self._ck(lbm_lib().lbm_init_case(self.h), "lbm_init_case")

    def geo(self) -> np.ndarray:
        """The reference mask codes of the local planes, int8 [nz][ny][nx]."""
        a = np.zeros(self.shape, np.int8)
        self._ck(lbm_lib().lbm_get_geo(self.h, _ptr(a, C.c_int8)), "lbm_get_geo")
        return a

    def set_f(self, f: np.ndarray):
        a = np.ascontiguousarray(f, np.float32)
        self._ck(lbm_lib().lbm_set_f(self.h, _ptr(a, C.c_float)), "lbm_set_f")

    def set_residual_order(self, mode=LBM_SUM_CUB_TREE, items_per_thread=16, vec=4, grid_cap=240):
        """lbm_set_residual_order: LBM_SUM_FP64 (the default) or LBM_SUM_CUB_TREE (the reference's
        storage order, thrust::reduce's CUB tree in fp32)."""
        self._ck(lbm_lib().lbm_set_residual_order(self.h, mode, items_per_thread, vec, grid_cap),
                 "lbm_set_residual_order")

    def set_convergence(self, enabled=True, max_it=10000, stag_max=50, tol=1e-6):
        self._ck(lbm_lib().lbm_set_convergence(self.h, 1 if enabled else 0, max_it, stag_max, tol),
                 "lbm_set_convergence")

    def step(self, n: int, history: bool = True):
        if not history:
            self._ck(lbm_lib().lbm_step(self.h, n, None, None), "lbm_step")
            return None
        hist = np.zeros(max(n, 1), np.float32)
        done = C.c_int(0)
        self._ck(lbm_lib().lbm_step(self.h, n, _ptr(hist, C.c_float), C.byref(done)), "lbm_step")
        return hist[:n]

    def sync(self):
        self._ck(lbm_lib().lbm_sync(self.h), "lbm_sync")

    def state(self):
        k, tc, st = C.c_int(), C.c_int(), C.c_int()
        r, s = C.c_float(), C.c_double()
        self._ck(lbm_lib().lbm_get_state(self.h, C.byref(k), C.byref(tc), C.byref(st), C.byref(r), C.byref(s)),
                 "lbm_get_state")
        nf = C.c_int()
        self._ck(lbm_lib().lbm_get_nonfinite(self.h, C.byref(nf)), "lbm_get_nonfinite")
        return {"k": k.value, "tol_count": tc.value, "stopped": st.value, "residual": r.value,
                "velsum": s.value, "nonfinite_k": nf.value}

    def macros(self):
        out = [np.zeros(self.shape, np.float32) for _ in range(4)]
        self._ck(lbm_lib().lbm_get_macros(self.h, *[_ptr(a, C.c_float) for a in out]), "lbm_get_macros")
        return tuple(out)

    def digest(self) -> np.ndarray:
        """Per-plane uint64 digest of the fluid (rho, u) bits keyed by global coordinates
        (lbm_field_digest): equal for bit-identical fields whatever the slab cut."""
        a = np.zeros(self.shape[0], np.uint64)
        self._ck(lbm_lib().lbm_field_digest(self.h, _ptr(a, C.c_uint64)), "lbm_field_digest")
        return a

    def f(self) -> np.ndarray:
        a = np.zeros((19,) + self.shape, np.float32)
        self._ck(lbm_lib().lbm_get_f(self.h, _ptr(a, C.c_float)), "lbm_get_f")
        return a

    def checkpoint_save(self, path: str) -> None:
        """The complete lattice state to a file (lbm_checkpoint_save)."""
        self._ck(lbm_lib().lbm_checkpoint_save(self.h, os.fsencode(path)), "lbm_checkpoint_save")

    def checkpoint_load(self, path: str) -> None:
        """Resume from lbm_checkpoint_save's file (same descriptor; lbm_checkpoint_load)."""
        self._ck(lbm_lib().lbm_checkpoint_load(self.h, os.fsencode(path)), "lbm_checkpoint_load")

    def counts(self):
        nb, nf, by = C.c_int64(), C.c_int64(), C.c_double()
        self._ck(lbm_lib().lbm_get_counts(self.h, C.byref(nb), C.byref(nf), C.byref(by)), "lbm_get_counts")
        ns = C.c_int64()
        self._ck(lbm_lib().lbm_get_boundary_cells(self.h, C.byref(ns)), "lbm_get_boundary_cells")
        return {"n_box": nb.value, "n_fluid": nf.value, "algo_bytes_per_step": by.value, "n_boundary": ns.value}

    def layout(self):
        """Device layout lbm_create chose: row axis (1 x, 2 y), row pitch, x_align (1..4),
        256-cell chunks holding fluid."""
        ra, pitch, xa, nch = C.c_int(), C.c_int(), C.c_int(), C.c_int64()
        self._ck(lbm_lib().lbm_get_layout(self.h, C.byref(ra), C.byref(pitch), C.byref(xa), C.byref(nch)),
                 "lbm_get_layout")
        return {"row_axis": ra.value, "pitch": pitch.value, "x_align": xa.value, "active_chunks": nch.value}

    def storage(self):
        """Population storage: compact rows or the dense box, cell slots per buffer, bytes of both."""
        cm, cells, by = C.c_int(), C.c_int64(), C.c_int64()
        self._ck(lbm_lib().lbm_get_storage(self.h, C.byref(cm), C.byref(cells), C.byref(by)), "lbm_get_storage")
        return {"compact": bool(cm.value), "cells": cells.value, "bytes": by.value}

    def nee_path(self):
        """How the step produces its NEE values (lbm_get_nee_path): "cells" (one-cell waves or
        none), "blocks", "fix" (k_nee_fix) or "records", and the most records one chunk holds."""
        p, m = C.c_int(), C.c_int()
        self._ck(lbm_lib().lbm_get_nee_path(self.h, C.byref(p), C.byref(m)), "lbm_get_nee_path")
        return {"path": ("cells", "blocks", "fix", "records")[p.value], "max_records": m.value}

    def setup_cost(self):
        """lbm_create's wall seconds, the device bytes the context holds and the most it held
        during creation (placement candidates), from hipMemGetInfo (lbm_get_setup_cost)."""
        s, b, pk = C.c_double(), C.c_int64(), C.c_int64()
        self._ck(lbm_lib().lbm_get_setup_cost(self.h, C.byref(s), C.byref(b), C.byref(pk)), "lbm_get_setup_cost")
        return {"create_s": round(s.value, 3), "device_bytes": b.value, "peak_bytes": pk.value}

    def launch_shape(self):
        """How the step kernel covers the chunks: cells per lane, chunk workgroups, whether they
        loop over their XCD's chunks (grid stride), mean share of busy chunk lanes."""
        cpl, mb, gs, fill = C.c_int(), C.c_int(), C.c_int(), C.c_double()
        self._ck(lbm_lib().lbm_get_launch_shape(self.h, C.byref(cpl), C.byref(mb), C.byref(gs), C.byref(fill)),
                 "lbm_get_launch_shape")
        return {"cells_per_lane": cpl.value, "main_blocks": mb.value, "grid_stride": gs.value,
                "lane_fill": round(fill.value, 3)}

    def numerics(self):
        """(fast_div in use, chunk waves that took the exact division since creation)."""
        fd, n = C.c_int(), C.c_int64()
        self._ck(lbm_lib().lbm_get_numerics(self.h, C.byref(fd), C.byref(n)), "lbm_get_numerics")
        return {"fast_div": bool(fd.value), "retried_chunks": n.value}

    def placement(self):
        """Population-buffer placement (lbm_buffer_placement): candidates' write rates (GB/s) and
        the two kept; an empty list when the first two allocations were taken unprobed."""
        gbs, n, ch = (C.c_double * 256)(), C.c_int(), (C.c_int * 2)()
        self._ck(lbm_lib().lbm_buffer_placement(self.h, gbs, 256, C.byref(n), ch), "lbm_buffer_placement")
        return {"candidate_write_gbs": [round(gbs[i], 1) for i in range(min(n.value, 256))], "chosen": [ch[0], ch[1]]}

    def profile(self, enabled=True):
        """lbm_profile: True / 1 per-launch HIP events, 2 one event pair per lbm_step call
        (spans: stats()["span_ms"] over stats()["span_launches"] steps), False / 0 off."""
        mode = 1 if enabled is True else 0 if enabled is False else int(enabled)
        self._ck(lbm_lib().lbm_profile(self.h, mode), "lbm_profile")

    def stats(self):
        ms, n, by = C.c_double(), C.c_int64(), C.c_double()
        self._ck(lbm_lib().lbm_stats(self.h, C.byref(ms), C.byref(n), C.byref(by)), "lbm_stats")
        out = {"kernel_ms": ms.value, "launches": n.value, "algo_bytes": by.value}
        for kind, name in ((0, "step_kernel"), (1, "step_kernel_src0"), (2, "step_kernel_src1"), (3, "edge"),
                           (4, "interior"), (5, "halo"), (6, "halo_exposed"), (7, "span")):
            m, k = C.c_double(), C.c_int64()
            self._ck(lbm_lib().lbm_kernel_times(self.h, kind, C.byref(m), C.byref(k)), "lbm_kernel_times")
            out[name + "_ms"], out[name + "_launches"] = m.value, k.value
        return out

    def comm_info(self):
        """(rank, communicator size) from RCCL (ncclCommCount); (0, 1) without RCCL."""
        r, n = C.c_int(), C.c_int()
        self._ck(lbm_lib().lbm_comm_info(self.h, C.byref(r), C.byref(n)), "lbm_comm_info")
        return r.value, n.value

    def debug_fail_next_wait(self):
        """Test hook: this context's next wait sees a failed RCCL peer (lbm_debug_fail_next_wait)."""
        self._ck(lbm_lib().lbm_debug_fail_next_wait(self.h), "lbm_debug_fail_next_wait")

    def debug_poison_walls(self):
        """Test hook: NaN into every wall cell's slots of both population buffers (lbm_debug_poison_walls)."""
        self._ck(lbm_lib().lbm_debug_poison_walls(self.h), "lbm_debug_poison_walls")

    def attach_rccl(self, uid: bytes, rank: int, nranks: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._ck(lbm_lib().lbm_attach_rccl(self.h, buf, rank, nranks), "lbm_attach_rccl")


# lbm_probe_stream_shapes' copy shapes, in order (lbm_kernels.hpp launch_probe_copy)
PROBE_SHAPES = ["grid_nt", "grid", "xcd_nt", "xcd", "xcd_nt_x2", "xcd_nt_x4", "xcd_nt_32k_blocks", "tiles_nt",
                "tiles", "tiles_ldsdma_nt", "tiles_ldsdma"]


def probe_stream_shapes(device: int = 0, nbytes: int = 8 << 30, reps: int = 5) -> dict:
    """Streaming-copy rate (read + write GB/s) of every copy shape (lbm_probe_stream_shapes)."""
    per = (C.c_double * 32)()
    n = C.c_int()
    rc = lbm_lib().lbm_probe_stream_shapes(device, nbytes, reps, per, 32, C.byref(n))
    if rc != 0:
        raise LbmError(f"lbm_probe_stream: {lbm_lib().lbm_last_error(None).decode()}")
    names = PROBE_SHAPES + [f"shape{i}" for i in range(len(PROBE_SHAPES), n.value)]
    return {names[i]: round(per[i], 1) for i in range(min(n.value, 32))}


def probe_stream(device: int = 0, nbytes: int = 8 << 30, reps: int = 5) -> float:
    """Best streaming-copy rate (read + write GB/s) of the device (lbm_probe_stream): the
    attainable HBM bandwidth next to the 8 TB/s spec peak."""
    return max(probe_stream_shapes(device, nbytes, reps).values())


def rccl_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    rc = lbm_lib().lbm_rccl_unique_id(buf)
    if rc != 0:
        raise LbmError(f"lbm_rccl_unique_id: {lbm_lib().lbm_last_error(None).decode()}")
    return bytes(buf)


def group_step(lats, n: int, history: bool = True):
    arr = (P * len(lats))(*[l.h for l in lats])
    hist = np.zeros(max(n, 1), np.float32) if history else None
    rc = lbm_lib().lbm_group_step(arr, len(lats), n, _ptr(hist, C.c_float))
    if rc != 0:
        raise LbmError(f"lbm_group_step: {lbm_lib().lbm_last_error(lats[0].h).decode()}")
    return None if hist is None else hist[:n]


def gpu_available() -> bool:
    return torch is not None and torch.cuda.is_available()


def require_gpu():
    if not gpu_available():
        raise LbmError("no HIP device visible: liblbm.so has no CPU fallback")
