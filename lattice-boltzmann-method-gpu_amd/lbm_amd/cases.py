"""The reference's three cases as liblbm contexts (host set-up through liblbm_host.so,
stepping through liblbm.so)."""
from __future__ import annotations

import os

import numpy as np

from . import (BIF_SHAPE, BIF_TAU, LBM_CASE_LDC, LBM_CASE_MASK, LBM_CASE_POISEUILLE, LBM_INIT_EXPANDED,
               LBM_INIT_LDC_WI, LDC_TAU, POIS_TAU, Lattice, geo_ldc, geo_mask, geo_poiseuille, initial_fields,
               lid_u, poiseuille_profile, read_bc_txt, read_geo_txt)

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIF_DIR = os.path.join(REPO, "tests", "golden", "bifurcation")


def ldc(nx: int, ny: int | None = None, nz: int | None = None, device: int = 0, tau: float = LDC_TAU):
    """ldc.cu: cavity box, lid on y = ny-2 moving along +z; wi-form initial state."""
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    geo = geo_ldc(nx, ny, nz)
    lat = Lattice(LBM_CASE_LDC, (nz, ny, nx), tau, geo, device=device)
    rho, ux, uy, uz = initial_fields(0, geo)
    lat.init_equilibrium(LBM_INIT_LDC_WI, rho, ux, uy, uz)
    return lat, geo


def ldc_device(nx: int, ny: int, nz: int, z_offset: int = 0, nz_global: int | None = None, device: int = 0,
               tau: float = LDC_TAU):
    """The same cavity generated on the device from global coordinates (a z-slab of a
    (nx, ny, nz_global) box starting at z_offset): the benchmark path, no host arrays."""
    lat = Lattice(LBM_CASE_LDC, (nz, ny, nx), tau, None, device=device, z_offset=z_offset,
                  nz_global=nz if nz_global is None else nz_global)
    lat.init_ldc()
    return lat


def poiseuille(nx: int, ny: int, nz: int, device: int = 0, tau: float = POIS_TAU):
    """Poiseulle.cu: pipe along y, parabolic velocity NEE at both ends, expanded-form init."""
    geo = geo_poiseuille(nx, ny, nz)
    prof = poiseuille_profile(nx, nz)
    lat = Lattice(LBM_CASE_POISEUILLE, (nz, ny, nx), tau, geo, inlet_uy=prof, outlet_uy=prof, device=device)
    rho, ux, uy, uz = initial_fields(1, geo)
    lat.init_equilibrium(LBM_INIT_EXPANDED, rho, ux, uy, uz)
    return lat, geo


def bifurcation(inlet_block: int = 0, geo_path: str | None = None, bc_path: str | None = None, device: int = 0):
    """bifurcation.cu: shipped geo.txt / bc.txt (inlet_block 0 = as shipped, 1 = the block that
    matches the shipped inlet cells)."""
    geo_path = geo_path or os.path.join(BIF_DIR, "geo.txt")
    bc_path = bc_path or os.path.join(BIF_DIR, "bc.txt")
    raw = read_geo_txt(geo_path, BIF_SHAPE)
    geo = geo_mask(raw)
    _, inl, outl = read_bc_txt(bc_path, geo, inlet_block)
    lat = Lattice(LBM_CASE_MASK, BIF_SHAPE, BIF_TAU, geo, inlet_uy=inl, device=device)
    rho, ux, uy, uz = initial_fields(2, geo, inl, outl)
    lat.init_equilibrium(LBM_INIT_EXPANDED, rho, ux, uy, uz)
    return lat, geo, inl, outl


def slab_bounds(nz_global: int, nslabs: int, i: int):
    """z range [z0, z1) of slab i of an even split (remainder to the lowest slabs)."""
    base, rem = divmod(nz_global, nslabs)
    z0 = i * base + min(i, rem)
    return z0, z0 + base + (1 if i < rem else 0)


def slab_geo(geo: np.ndarray, z0: int, z1: int) -> np.ndarray:
    """Planes z0-1 .. z1 of a global mask (one halo plane each side, 0 outside the box)."""
    nz, ny, nx = geo.shape
    out = np.zeros((z1 - z0 + 2, ny, nx), np.int8)
    for k, z in enumerate(range(z0 - 1, z1 + 1)):
        if 0 <= z < nz:
            out[k] = geo[z]
    return out
