"""Host ingest (liblbm_host.so, the per-case set-up of the reference) against the oracle's
independent restatement and the reference's own data files.  CPU only."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

BIF = os.path.join(GOLDEN, "bifurcation")


@pytest.mark.parametrize("shape", [(16, 16, 16), (12, 20, 9), (64, 64, 64)])
def test_geo_ldc_matches_oracle(lbm, oracle, shape):
    nx, ny, nz = shape
    assert np.array_equal(lbm.geo_ldc(nx, ny, nz), oracle.geo_ldc(nx, ny, nz))


@pytest.mark.parametrize("shape", [(20, 24, 20), (64, 64, 64), (33, 17, 33)])
def test_geo_poiseuille_matches_oracle(lbm, oracle, shape):
    nx, ny, nz = shape
    assert np.array_equal(lbm.geo_poiseuille(nx, ny, nz), oracle.geo_poiseuille(nx, ny, nz))


def test_bifurcation_mask_and_tables(lbm, oracle):
    raw = lbm.read_geo_txt(os.path.join(BIF, "geo.txt"))
    raw_o = oracle.read_geo_txt(os.path.join(BIF, "geo.txt"), 64, 83, 32)
    assert np.array_equal(raw, raw_o)
    geo = lbm.geo_mask(raw)
    assert np.array_equal(geo, oracle.geo_mask(raw_o))
    for block in (0, 1):
        n, inl, outl = lbm.read_bc_txt(os.path.join(BIF, "bc.txt"), geo, block)
        n_o, inl_o, outl_o = oracle.read_bc_txt(os.path.join(BIF, "bc.txt"), geo, block)
        assert n == n_o
        assert np.array_equal(inl.view(np.uint32), inl_o.view(np.uint32))
        assert np.array_equal(outl.view(np.uint32), outl_o.view(np.uint32))
        # unmasked tables (device mask path): equal to the masked ones on the coded cells
        n_u, inl_u, outl_u = lbm.read_bc_txt(os.path.join(BIF, "bc.txt"), geo.shape, block)
        assert n_u == n
        assert np.array_equal(np.where(geo[:, 1, :] == 2, inl_u, 0), inl)
        assert np.array_equal(np.where(geo[:, -2, :] == 3, outl_u, 0), outl)


def test_slab_mask_planes(lbm):
    """slab_mask: the halo slab's raw planes z0-3 .. z1+2, zero outside the box."""
    from lbm_amd import cases
    raw = np.arange(5 * 6 * 7).reshape(5, 6, 7).astype(np.uint8)
    m = cases.slab_mask(raw, 1, 3)
    assert m.shape == (8, 6, 7)
    assert not m[:2].any() and np.array_equal(m[2:7], raw) and not m[7].any()


def test_known_answers(lbm):
    """SURVEY.md 8(c) known answers: NLATTICE of the Poiseuille pipe (214128) and of the
    bifurcation (65820, thesis 4.8), its class counts, and 6144 tokens in bc.txt."""
    n, _ = lbm.index_transform(lbm.geo_poiseuille(64, 64, 64))
    assert n == 214128
    assert int((lbm.geo_poiseuille(64, 64, 64) == 4).sum()) == 175200
    geo = lbm.geo_mask(lbm.read_geo_txt(os.path.join(BIF, "geo.txt")))
    n, idx = lbm.index_transform(geo)
    assert n == 65820
    counts = {int(k): int(v) for k, v in zip(*np.unique(geo, return_counts=True))}
    assert counts == {-1: 12214, 0: 104164, 1: 7648, 2: 345, 3: 306, 4: 45307}
    assert idx.max() == n - 1 and (idx >= 0).sum() == n
    tokens = open(os.path.join(BIF, "bc.txt")).read().split()
    assert len(tokens) == 6144


def test_index_transform_matches_oracle(lbm, oracle):
    for geo in (lbm.geo_poiseuille(20, 24, 20), lbm.geo_ldc(10, 11, 12)):
        n, idx = lbm.index_transform(geo)
        n_o, idx_o = oracle.index_transform(geo)
        assert n == n_o and np.array_equal(idx, idx_o)


def test_poiseuille_profile(lbm):
    """uygt of Poiseulle.cu:590,597: u_max (1 - ((x-cx)^2 + (z-cz)^2) / r^2) in fp32."""
    nx, nz = 20, 20
    t = lbm.poiseuille_profile(nx, nz)
    c = np.float32((nx - 1) / 2.0)
    cz = np.float32((nz - 1) / 2.0)
    r = np.float32((nx - 1) / 2.0)
    x = np.arange(nx, dtype=np.float32)[None, :]
    z = np.arange(nz, dtype=np.float32)[:, None]
    um = np.float32(lbm.POIS_UMAX_KERNEL)
    want = um * (np.float32(1.0) - ((x - c) * (x - c) + (z - cz) * (z - cz)) / (r * r))
    assert np.array_equal(t.view(np.uint32), want.astype(np.float32).view(np.uint32))


def test_initial_fields(lbm):
    """initialize() fields: LDC lid rows (ldc.cu:510-532), Poiseuille parabola on the two
    end planes of stored cells (Poiseulle.cu:280-341), bifurcation tables (bifurcation.cu:333-373)."""
    g = lbm.geo_ldc(12, 14, 10)
    rho, ux, uy, uz = lbm.initial_fields(0, g)
    assert np.all(rho == 1) and not ux.any() and not uy.any()
    lid = np.float32(lbm.lid_u())
    assert np.all(uz[:, 12:14, :] == lid) and not uz[:, :12, :].any()
    g = lbm.geo_poiseuille(20, 24, 20)
    rho, ux, uy, uz = lbm.initial_fields(1, g)
    assert not ux.any() and not uz.any()
    ends = [0, 1, 22, 23]
    mid = np.setdiff1d(np.arange(24), ends)
    assert not uy[:, mid, :].any()
    assert np.all(uy[:, ends, :][g[:, ends, :] == 0] == 0)
    assert uy[:, ends, :].max() > 0
    geo = lbm.geo_mask(lbm.read_geo_txt(os.path.join(BIF, "geo.txt")))
    _, inl, outl = lbm.read_bc_txt(os.path.join(BIF, "bc.txt"), geo, 1)
    rho, ux, uy, uz = lbm.initial_fields(2, geo, inl, outl)
    stored = geo != 0
    assert np.array_equal(uy[:, 1, :][stored[:, 1, :]], inl[stored[:, 1, :]])
    assert np.array_equal(uy[:, 81, :][stored[:, 81, :]], outl[stored[:, 81, :]])


def test_vtk_format(lbm, tmp_path):
    """outputSave (ldc.cu:582-610): legacy ASCII VTK header, DIMENSIONS
    NX-4 NY-4 NZ-4 over x,y,z in [2, N-3], then every u*C_U value on one line (6 digits)."""
    nx, ny, nz = 10, 9, 8
    g = lbm.geo_ldc(nx, ny, nz)
    ux = np.full(g.shape, 0.5, np.float32)
    uy = np.zeros(g.shape, np.float32)
    uz = np.full(g.shape, -0.123456789, np.float32)
    p = tmp_path / "out.vtk"
    lbm.write_vtk(str(p), 0, g, ux, uy, uz, 2.0, 1.0)
    text = p.read_text().splitlines()
    assert text[0] == "# vtk DataFile Version 2.0"
    assert text[2:4] == ["ASCII", "DATASET STRUCTURED_POINTS"]
    assert text[4] == f"DIMENSIONS {nx - 4} {ny - 4} {nz - 4}"
    assert text[5] == "SPACING 1 1 1"
    assert text[6] == f"ORIGIN {nx // 2 - 1} {ny // 2 - 1} 0"
    n = (nx - 4) * (ny - 4) * (nz - 4)
    assert text[7].split() == ["POINT_DATA", str(n)]
    assert text[8] == "VECTORS VELOCITY float"
    vals = text[9].split()
    assert len(vals) == 3 * n
    assert vals[:3] == ["1", "0", "-0.246914"]


def test_calc_res_matches_oracle(lbm, oracle):
    raw = oracle.read_geo_txt(os.path.join(BIF, "geo.txt"), 64, 83, 32)
    geo = oracle.geo_mask(raw)
    _, inl, outl = oracle.read_bc_txt(os.path.join(BIF, "bc.txt"), geo, 1)
    o = oracle.Oracle(oracle.MASK, geo, 0.55, inlet_uy=inl, outlet_uy=outl)
    o.step(30)
    rho, ux, uy, uz = o.macros()
    assert lbm.calc_res(geo, ux, uy, uz) == pytest.approx(o.calc_res_bif(), rel=1e-12)
