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


def duct_generic(nx: int, ny: int, nz: int, u_in: float = 0.05, u_out: float = 0.045, u_side: float = 0.01):
    """A coronary-style test geometry for LBM_CASE_GENERIC (coronary.cu:716-944's boundary
    scheme on every kind of face): a duct along x with
      code 2  inlet at x = 1, face +x, velocity + rho = 1 (parabolic u_x table over y,z),
      code 3  outlet at x = nx-2, face -x, velocity with rho of the fluid,
      code 5  side outlet patch in the top wall z = nz-2, face -z, velocity (0, 0, u_side),
      code 6  pressure patch in the y = 1 wall, face +y, rho = 1, u of the fluid.
    Returns (geo [nz][ny][nx] int8, bc_codes list of dicts, initial (rho, ux, uy, uz))."""
    g = np.zeros((nz, ny, nx), np.int8)
    g[1:nz - 1, 1:ny - 1, 1:nx - 1] = 1
    g[2:nz - 2, 2:ny - 2, 2:nx - 2] = 4
    g[2:nz - 2, 2:ny - 2, 1] = 2
    g[2:nz - 2, 2:ny - 2, nx - 2] = 3
    cx, cy = nx // 2, ny // 2
    g[nz - 2, cy - 2:cy + 3, cx - 2:cx + 3] = 5
    g[3:6, 1, 4:7] = 6
    yy, zz = np.meshgrid(np.arange(ny, dtype=np.float32), np.arange(nz, dtype=np.float32))
    ry, rz = np.float32((ny - 5) / 2.0), np.float32((nz - 5) / 2.0)
    prof = np.float32(u_in) * (np.float32(1) - ((yy - np.float32((ny - 1) / 2)) / ry) ** 2) * \
        (np.float32(1) - ((zz - np.float32((nz - 1) / 2)) / rz) ** 2)
    prof = np.clip(prof, 0, None).astype(np.float32)  # [z][y]
    bcs = [
        {"code": 2, "face": 0, "kind": 1, "rho": 1.0, "u": (u_in, 0.0, 0.0), "table": prof},
        {"code": 3, "face": 1, "kind": 0, "u": (u_out, 0.0, 0.0)},
        {"code": 5, "face": 5, "kind": 0, "u": (0.0, 0.0, u_side)},
        {"code": 6, "face": 2, "kind": 2, "rho": 1.0},
    ]
    rho = np.where(g != 0, np.float32(1), np.float32(1)).astype(np.float32)
    ux = np.zeros(g.shape, np.float32)
    uy = np.zeros(g.shape, np.float32)
    uz = np.zeros(g.shape, np.float32)
    ux[g == 2] = prof[g[:, :, 1] == 2]
    ux[g == 3] = np.float32(u_out)
    uz[g == 5] = np.float32(u_side)
    return g, bcs, (rho, ux, uy, uz)


def generic(geo, bcs, fields, tau: float = 0.6, device: int = 0):
    """A LBM_CASE_GENERIC lattice initialised at the equilibrium of `fields` (expanded form)."""
    from . import LBM_CASE_GENERIC
    nz, ny, nx = geo.shape
    lat = Lattice(LBM_CASE_GENERIC, (nz, ny, nx), tau, geo, device=device, bc_codes=bcs)
    lat.init_equilibrium(LBM_INIT_EXPANDED, *fields)
    return lat


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


def slab_mask(raw: np.ndarray, z0: int, z1: int) -> np.ndarray:
    """Planes z0-3 .. z1+2 of a global raw mask, uint8 (lbm_desc.mask of a halo slab: geo_pre of
    the halo planes reads two planes beyond them); planes outside the box are zero."""
    nz, ny, nx = raw.shape
    out = np.zeros((z1 - z0 + 6, ny, nx), np.uint8)
    for k, z in enumerate(range(z0 - 3, z1 + 3)):
        if 0 <= z < nz:
            out[k] = raw[z]
    return out


def mask_device(raw: np.ndarray, inlet_uy=None, outlet_uy=None, tau: float = BIF_TAU, device: int = 0,
                z_offset: int = 0, nz_global: int | None = None, halo_planes: bool = False, x_align: int = 0):
    """bifurcation.cu's set-up with geo_pre on the device: `raw` is the geo.txt
    mask (uint8; with halo_planes the slab_mask of this slab), the codes are built and the
    initial state is evaluated on the device (lbm_init_case).  inlet_uy / outlet_uy are the
    bc.txt tables, masked or not."""
    m = np.ascontiguousarray(raw, np.uint8)
    nz = m.shape[0] - (6 if halo_planes else 0)
    lat = Lattice(LBM_CASE_MASK, (nz, m.shape[1], m.shape[2]), tau, None, mask=m, inlet_uy=inlet_uy,
                  outlet_uy=outlet_uy, device=device, z_offset=z_offset, nz_global=nz_global,
                  halo_planes=halo_planes, x_align=x_align)
    lat.init_case()
    return lat


def bifurcation_device(inlet_block: int = 0, geo_path: str | None = None, bc_path: str | None = None,
                       device: int = 0):
    """bifurcation() with the mask codes built and the state initialised on the device."""
    geo_path = geo_path or os.path.join(BIF_DIR, "geo.txt")
    bc_path = bc_path or os.path.join(BIF_DIR, "bc.txt")
    raw = read_geo_txt(geo_path, BIF_SHAPE)
    _, inl, outl = read_bc_txt(bc_path, tuple(BIF_SHAPE), inlet_block)
    return mask_device(raw.astype(np.uint8), inl, outl, device=device), raw


def bifurcation_upsampled(k: int = 4, inlet_block: int = 1, geo_path: str | None = None,
                          bc_path: str | None = None, device: int = 0):
    """SURVEY 8(d) C4's bandwidth-relevant sparse variant: the shipped geo.txt mask nearest-
    upsampled k times along every axis (k = 4: 256 x 332 x 128, ~4 M stored cells) and bc.txt's
    inlet / outlet tables with it; geo_pre and initialize() on the device.  The default inlet
    is block 1 (the block whose inlet drives a flow through the tree).  Returns (lat, raw)."""
    geo_path = geo_path or os.path.join(BIF_DIR, "geo.txt")
    bc_path = bc_path or os.path.join(BIF_DIR, "bc.txt")
    raw = read_geo_txt(geo_path, BIF_SHAPE).astype(np.uint8)
    _, inl, outl = read_bc_txt(bc_path, tuple(BIF_SHAPE), inlet_block)
    up = np.ascontiguousarray(raw.repeat(k, 0).repeat(k, 1).repeat(k, 2))
    big = [np.ascontiguousarray(t.repeat(k, 0).repeat(k, 1)) for t in (inl, outl)]
    return mask_device(up, big[0], big[1], device=device), up


def coronary_bc_codes(c_u: float = 2.74909090909091):
    """The boundary codes of coronary.cu's boundary_stream (716-944) as LBM_CASE_GENERIC entries:
    code 2 inlet (fluid at x+1): u_bc = (0.1745/C_U, 0, 0), rho_bc = 1;
    code 3 outlet (fluid at x-1): u_bc = (0.1/C_U, 0, 0), rho of the fluid neighbour;
    codes 5, 6, 7 outlets (fluid at z-1): u_bc = (0, 0, 0.02/C_U), rho of the fluid neighbour.
    The velocities are the reference's double quotients rounded to float.  Each outgoing
    population gets its own NEE value from its own fluid neighbour and equilibrium (the code-3
    branch, coronary.cu:795-867, writes slots 2, 9, 10, 13 and 14 that way)."""
    from . import LBM_BC_VELOCITY, LBM_BC_VELOCITY_RHO, LBM_FACE_NX, LBM_FACE_NZ, LBM_FACE_PX
    cu = np.float32(c_u)
    uin = float(np.float32(0.1745 / float(cu)))
    uout = float(np.float32(0.1 / float(cu)))
    uz = float(np.float32(0.02 / float(cu)))
    codes = [{"code": 2, "face": LBM_FACE_PX, "kind": LBM_BC_VELOCITY_RHO, "rho": 1.0, "u": (uin, 0.0, 0.0)},
             {"code": 3, "face": LBM_FACE_NX, "kind": LBM_BC_VELOCITY, "u": (uout, 0.0, 0.0)}]
    codes += [{"code": k, "face": LBM_FACE_NZ, "kind": LBM_BC_VELOCITY, "u": (0.0, 0.0, uz)} for k in (5, 6, 7)]
    return codes


# coronary_cfd/coronary.cu: box, relaxation time and output constants (coronary.cu:19-20, 23, 357)
CORONARY_SHAPE = (372, 291, 291)  # (nz, ny, nx)
CORONARY_TAU = 0.55
CORONARY_C_U, CORONARY_CH, CORONARY_C_RHO = 2.74909090909091, 6.1111e-05, 1060.0


def vessel_mask(shape, tube, branches):
    """A synthetic vessel tree as a raw 0/1 mask (the reference's coronary geo.txt is not shipped):
    tube = (x0, x1, yc, zc, r): a main vessel along x over [x0, x1] with a circular cross-section;
    branches = [(xc, yc, z0, z1, r)]: vessels along z over [z0, z1].  Open ends sit where a
    vessel stops: the planes x = x0, x = x1 and z = z1 of each branch."""
    nz, ny, nx = shape
    raw = np.zeros(shape, np.int32)
    z, y, x = np.ogrid[:nz, :ny, :nx]
    x0, x1, yc, zc, r = tube
    raw[((y - yc) ** 2 + (z - zc) ** 2 <= r * r) & (x >= x0) & (x <= x1)] = 1
    for xc, byc, z0, z1, br in branches:
        raw[((x - xc) ** 2 + (y - byc) ** 2 <= br * br) & (z >= z0) & (z <= z1)] = 1
    return raw


def coronary_reference_vessel():
    """A vessel tree in the reference's 291 x 291 x 372 box whose open ends lie on coronary.cu's
    five end planes, inside their windows: main vessel x = 3 .. 272 (inlet, main exit), branches
    ending at z = 185 (window x 217..236, y 113..137), 191 (x 160..205, y 159..199) and 204."""
    return vessel_mask(CORONARY_SHAPE, (3, 272, 150, 60, 30),
                       [(227, 125, 60, 185, 6), (183, 179, 60, 191, 8), (100, 150, 60, 204, 10)])


def coronary_small_vessel():
    """A small vessel tree with its own end table (same roles and pass counts as coronary.cu's
    ends): inlet x = 3, main exit x = 50, branches ending at z = 30 / 33 (windows) and z = 36
    (whole plane).  Returns (raw, ends)."""
    shape = (40, 28, 56)
    raw = vessel_mask(shape, (3, 50, 14, 12, 8), [(20, 14, 12, 30, 3), (36, 12, 12, 33, 3), (44, 16, 12, 36, 3)])
    nz, ny, nx = shape
    ends = [(0, 3, 1, ny - 1, 1, nz - 1, 1), (0, 50, 1, ny - 1, 1, nz - 1, 2), (2, 30, 15, 26, 9, 20, 4),
            (2, 33, 31, 42, 7, 18, 5), (2, 36, 1, nx - 1, 1, ny - 1, 6)]
    return raw, ends


def coronary(raw: np.ndarray, ends=None, device: int = 0, tau: float = CORONARY_TAU):
    """coronary.cu's set-up as a LBM_CASE_GENERIC lattice: geo_pre of the raw vessel mask with
    its open ends (the reference's five for its box by default), the coronary boundary codes
    (coronary_bc_codes) and initialize()'s state (coronary.cu:277-350).  Returns (lat, geo)."""
    from . import LBM_CASE_GENERIC, coronary_ends, geo_ends
    geo = geo_ends(raw, coronary_ends(raw.shape) if ends is None else ends)
    lat = Lattice(LBM_CASE_GENERIC, geo.shape, tau, geo, device=device, bc_codes=coronary_bc_codes())
    lat.init_equilibrium(LBM_INIT_EXPANDED, *initial_fields(3, geo))
    return lat, geo
