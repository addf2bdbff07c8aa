"""ctypes wrapper of the CPU oracle (oracle/liblbm_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblbm_oracle.so")

LDC, POISEUILLE, MASK, GENERIC = 0, 1, 2, 3


class orc_bc(C.Structure):
    _fields_ = [("code", C.c_int), ("face", C.c_int), ("kind", C.c_int), ("rho", C.c_float),
                ("u", C.c_float * 3), ("table", C.POINTER(C.c_float))]
TWO_PHASE, SERIAL_EMU = 0, 1

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < max(
        os.path.getmtime(os.path.join(HERE, f)) for f in ("lbm_oracle.c", "lbm_oracle.h", "Makefile")
    ):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        i8p, i32p, f32p = C.POINTER(C.c_int8), C.POINTER(C.c_int32), C.POINTER(C.c_float)
        sig = {
            "orc_geo_ldc": (None, [C.c_int, C.c_int, C.c_int, i8p]),
            "orc_geo_poiseuille": (None, [C.c_int, C.c_int, C.c_int, i8p]),
            "orc_geo_mask": (None, [C.c_int, C.c_int, C.c_int, i32p, i8p]),
            "orc_read_geo_txt": (C.c_int, [C.c_char_p, C.c_int, i32p]),
            "orc_read_geo_txt_zxy": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, i32p]),
            "orc_geo_coronary": (None, [C.c_int, C.c_int, C.c_int, i32p, C.c_int, i32p, i8p]),
            "orc_read_bc_txt": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, i8p, C.c_int, f32p, f32p]),
            "orc_index_transform": (C.c_int, [C.c_int, C.c_int, C.c_int, i8p, i32p]),
            "orc_create": (P, [C.c_int, C.c_int, C.c_int, C.c_int, i8p, C.c_float, C.c_int, f32p, f32p]),
            "orc_destroy": (None, [P]),
            "orc_create_generic": (P, [C.c_int, C.c_int, C.c_int, i8p, C.c_float, C.POINTER(orc_bc), C.c_int]),
            "orc_feq": (None, [C.c_float, C.c_float, C.c_float, C.c_float, f32p]),
            "orc_feq_bc": (None, [C.c_float, C.c_float, C.c_float, C.c_float, f32p]),
            "orc_initialize": (None, [P]),
            "orc_initialize_coronary": (None, [P]),
            "orc_step": (None, [P, C.c_int, f32p]),
            "orc_run_converge": (C.c_int, [P, C.c_int, C.c_int, C.c_float, f32p]),
            "orc_steps_done": (C.c_int, [P]),
            "orc_get_macros": (None, [P, f32p, f32p, f32p, f32p]),
            "orc_get_f": (None, [P, f32p]),
            "orc_set_f": (None, [P, f32p]),
            "orc_bad_reads": (C.c_long, [P]),
            "orc_calc_res_bif": (C.c_double, [P]),
            "orc_velsum": (C.c_float, [P]),
            "orc_set_residual_fp64": (None, [P, C.c_int]),
            "orc_set_residual_mode": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int]),
            "orc_cub_reduce": (C.c_float, [f32p, C.c_long, C.c_int, C.c_int, C.c_int]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(C.POINTER(ct))


def geo_ldc(nx: int, ny: int, nz: int) -> np.ndarray:
    g = np.zeros((nz, ny, nx), np.int8)
    lib().orc_geo_ldc(nx, ny, nz, _p(g, C.c_int8))
    return g


def geo_poiseuille(nx: int, ny: int, nz: int) -> np.ndarray:
    g = np.zeros((nz, ny, nx), np.int8)
    lib().orc_geo_poiseuille(nx, ny, nz, _p(g, C.c_int8))
    return g


def read_geo_txt(path: str, nx: int, ny: int, nz: int) -> np.ndarray:
    raw = np.zeros((nz, ny, nx), np.int32)
    n = lib().orc_read_geo_txt(path.encode(), raw.size, _p(raw, C.c_int32))
    if n != raw.size:
        raise ValueError(f"{path}: read {n} of {raw.size} ints")
    return raw


def geo_mask(raw: np.ndarray) -> np.ndarray:
    nz, ny, nx = raw.shape
    raw = np.ascontiguousarray(raw, np.int32)
    g = np.zeros((nz, ny, nx), np.int8)
    lib().orc_geo_mask(nx, ny, nz, _p(raw, C.c_int32), _p(g, C.c_int8))
    return g


def read_geo_txt_zxy(path: str, nx: int, ny: int, nz: int) -> np.ndarray:
    """coronary.cu:45-56: geo.txt in z, x, y loop order, returned as a raster [nz][ny][nx]."""
    raw = np.zeros((nz, ny, nx), np.int32)
    n = lib().orc_read_geo_txt_zxy(path.encode(), nx, ny, nz, _p(raw, C.c_int32))
    if n != raw.size:
        raise ValueError(f"{path}: read {n} of {raw.size} ints")
    return raw


def coronary_ends(nx: int, ny: int, nz: int):
    """The five ends coronary.cu:75-143 hard-codes for its 291 x 291 x 372 box, as
    (axis, plane, lo0, hi0, lo1, hi1, passes): x = 3 over y, z in [1, N-2] once (inlet, code 2);
    x = 272 twice (3); z = 185 over x in [217, 237), y in [113, 138) four times (5); z = 191 over
    x in [160, 206), y in [159, 200) five times (6); z = 204 over x, y in [1, N-2] six times (7)."""
    return [(0, 3, 1, ny - 1, 1, nz - 1, 1), (0, 272, 1, ny - 1, 1, nz - 1, 2),
            (2, 185, 217, 237, 113, 138, 4), (2, 191, 160, 206, 159, 200, 5),
            (2, 204, 1, nx - 1, 1, ny - 1, 6)]


def geo_coronary(raw: np.ndarray, ends) -> np.ndarray:
    """coronary.cu:31-275 geo_pre with the end table `ends` (coronary_ends for the reference box)."""
    nz, ny, nx = raw.shape
    raw = np.ascontiguousarray(raw, np.int32)
    e = np.ascontiguousarray(np.array(ends, np.int32).reshape(-1))
    g = np.zeros((nz, ny, nx), np.int8)
    lib().orc_geo_coronary(nx, ny, nz, _p(raw, C.c_int32), len(ends), _p(e, C.c_int32), _p(g, C.c_int8))
    return g


def read_bc_txt(path: str, geo: np.ndarray, skip_blocks: int = 0):
    nz, ny, nx = geo.shape
    inl = np.zeros((nz, nx), np.float32)
    out = np.zeros((nz, nx), np.float32)
    n = lib().orc_read_bc_txt(path.encode(), nx, ny, nz, _p(geo, C.c_int8), skip_blocks,
                              _p(inl, C.c_float), _p(out, C.c_float))
    return n, inl, out


def index_transform(geo: np.ndarray):
    nz, ny, nx = geo.shape
    idx = np.zeros(geo.shape, np.int32)
    n = lib().orc_index_transform(nx, ny, nz, _p(geo, C.c_int8), _p(idx, C.c_int32))
    return n, idx


class Oracle:
    """Serial CPU restatement of one reference case."""

    def __init__(self, kind: int, geo: np.ndarray, tau: float, ldc_order: int = TWO_PHASE,
                 inlet_uy: np.ndarray | None = None, outlet_uy: np.ndarray | None = None, bcs=None):
        self.geo = np.ascontiguousarray(geo, np.int8)
        self.nz, self.ny, self.nx = self.geo.shape
        self.kind = kind
        self._keep = []
        ip = op = None
        if inlet_uy is not None:
            a = np.ascontiguousarray(inlet_uy, np.float32); self._keep.append(a); ip = _p(a, C.c_float)
        if outlet_uy is not None:
            a = np.ascontiguousarray(outlet_uy, np.float32); self._keep.append(a); op = _p(a, C.c_float)
        if kind == GENERIC:
            arr = (orc_bc * max(1, len(bcs or [])))()
            for k, b in enumerate(bcs or []):
                arr[k].code, arr[k].face, arr[k].kind = b["code"], b["face"], b["kind"]
                arr[k].rho = b.get("rho", 1.0)
                for i, v in enumerate(b.get("u", (0.0, 0.0, 0.0))):
                    arr[k].u[i] = v
                if b.get("table") is not None:
                    t = np.ascontiguousarray(b["table"], np.float32)
                    self._keep.append(t)
                    arr[k].table = _p(t, C.c_float)
            self.h = lib().orc_create_generic(self.nx, self.ny, self.nz, _p(self.geo, C.c_int8), float(tau), arr,
                                              len(bcs or []))
        else:
            self.h = lib().orc_create(kind, self.nx, self.ny, self.nz, _p(self.geo, C.c_int8), float(tau),
                                      ldc_order, ip, op)
        lib().orc_initialize(self.h)

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            _lib.orc_destroy(h)
            self.h = None

    @property
    def ncell(self) -> int:
        return self.nx * self.ny * self.nz

    def step(self, n: int) -> np.ndarray:
        hist = np.zeros(max(n, 1), np.float32)
        lib().orc_step(self.h, n, _p(hist, C.c_float))
        return hist[:n]

    def run_converge(self, max_it=10000, stag_max=50, tol=1e-6):
        r = np.zeros(1, np.float32)
        k = lib().orc_run_converge(self.h, max_it, stag_max, tol, _p(r, C.c_float))
        return k, float(r[0])

    def macros(self):
        shp = (self.nz, self.ny, self.nx)
        out = [np.zeros(shp, np.float32) for _ in range(4)]
        lib().orc_get_macros(self.h, *[_p(a, C.c_float) for a in out])
        return tuple(out)  # rho, ux, uy, uz

    def f(self) -> np.ndarray:
        a = np.zeros((19, self.nz, self.ny, self.nx), np.float32)
        lib().orc_get_f(self.h, _p(a, C.c_float))
        return a

    def set_f(self, f: np.ndarray) -> None:
        a = np.ascontiguousarray(f, np.float32)
        lib().orc_set_f(self.h, _p(a, C.c_float))

    def initialize_coronary(self) -> None:
        """Replace the generic initial state with coronary.cu:277-350's (float velocity quotients)."""
        lib().orc_initialize_coronary(self.h)

    def bad_reads(self) -> int:
        return int(lib().orc_bad_reads(self.h))

    def calc_res_bif(self) -> float:
        return float(lib().orc_calc_res_bif(self.h))

    def velsum(self) -> float:
        return float(lib().orc_velsum(self.h))

    def residual_fp64(self, on: bool = True) -> None:
        """Sum |u| in fp64 like liblbm (default: thrust's fp32 sum, serial, storage order)."""
        lib().orc_set_residual_fp64(self.h, 1 if on else 0)

    def residual_cub_tree(self, ipt: int = 16, vec: int = 4, grid_cap: int = 240) -> None:
        """Sum |u| with thrust::reduce's CUB two-pass fp32 tree (orc_cub_reduce)."""
        if lib().orc_set_residual_mode(self.h, SUM_CUB_TREE, ipt, vec, grid_cap) != 0:
            raise ValueError(f"bad CUB tree parameters ipt={ipt} vec={vec} grid_cap={grid_cap}")


SUM_SERIAL, SUM_FP64, SUM_CUB_TREE = 0, 1, 2


def cub_reduce(v: np.ndarray, ipt: int = 16, vec: int = 4, grid_cap: int = 240) -> float:
    """orc_cub_reduce over a float32 array (the emulated CUB two-pass tree)."""
    v = np.ascontiguousarray(v, np.float32)
    return float(lib().orc_cub_reduce(_p(v, C.c_float), v.size, ipt, vec, grid_cap))


def feq(rho: float, ux: float, uy: float, uz: float) -> np.ndarray:
    """The update kernel's equilibrium (Poiseulle.cu:561-580) in fp32."""
    out = np.zeros(19, np.float32)
    lib().orc_feq(rho, ux, uy, uz, _p(out, C.c_float))
    return out


def feq_bc(rho: float, ux: float, uy: float, uz: float) -> np.ndarray:
    """The NEE boundary-value equilibrium (the reference's fp32 tmp terms)."""
    out = np.zeros(19, np.float32)
    lib().orc_feq_bc(rho, ux, uy, uz, _p(out, C.c_float))
    return out


# reference per-case constants (ldc.cu:48-55, Poiseulle.cu:38-44, bifurcation.cu:19-20,434)
TAU = {LDC: 0.55, POISEUILLE: 0.58, MASK: 0.55}
