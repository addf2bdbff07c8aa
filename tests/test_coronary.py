"""coronary_cfd/coronary.cu's set-up on the host: geo.txt in z, x, y order
(coronary.cu:45-56), geo_pre with the five open ends (31-275), initialize()'s velocities
(277-350) and outputSave's three-section VTK (948-1011) -- liblbm_host.so against the oracle's
line-by-line restatement (oracle/lbm_oracle.c orc_geo_coronary) and against writers written
here from the reference text.  The reference's own geo.txt is not shipped, so the geometries are
synthetic vessel trees whose ends lie on the reference's end planes (cases.coronary_*_vessel)."""
import numpy as np
import pytest

f32 = np.float32


def test_coronary_end_table(lbm, oracle):
    from lbm_amd import cases
    assert lbm.coronary_ends(cases.CORONARY_SHAPE) == [tuple(e) for e in oracle.coronary_ends(291, 291, 372)]
    with pytest.raises(lbm.LbmError):
        lbm.coronary_ends((40, 28, 56))


def test_geo_ends_small_vs_oracle(lbm, oracle):
    from lbm_amd import cases
    raw, ends = cases.coronary_small_vessel()
    g = lbm.geo_ends(raw, ends)
    assert np.array_equal(g, oracle.geo_coronary(raw, ends))
    # every end code sits on its own plane only, and has fluid behind it
    for (axis, plane, *_r, passes) in ends:
        code = 1 + passes
        zz, yy, xx = np.nonzero(g == code)
        assert zz.size > 0
        assert np.all((xx if axis == 0 else zz) == plane), code
    zz, yy, xx = np.nonzero(g == 2)
    assert np.all(g[zz, yy, xx + 1] == 4)
    zz, yy, xx = np.nonzero(g == 5)
    assert np.all(g[zz - 1, yy, xx] == 4)


def test_geo_ends_rejects_ends_outside_the_interior(lbm):
    from lbm_amd import cases
    raw, ends = cases.coronary_small_vessel()
    nz, ny, nx = raw.shape
    for bad in [(0, 0, 1, ny - 1, 1, nz - 1, 1), (2, nz - 1, 1, nx - 1, 1, ny - 1, 1), (0, 3, 0, ny - 1, 1, nz - 1, 1),
                (2, 30, 1, nx, 1, ny - 1, 4), (1, 5, 1, 5, 1, 5, 1)]:
        with pytest.raises(lbm.LbmError):
            lbm.geo_ends(raw, [bad])


def test_geo_ends_reference_box_vs_oracle(lbm, oracle):
    from lbm_amd import cases
    raw = cases.coronary_reference_vessel()
    g = lbm.geo_ends(raw, lbm.coronary_ends(raw.shape))
    go = oracle.geo_coronary(raw, oracle.coronary_ends(291, 291, 372))
    assert np.array_equal(g, go)
    counts = {int(k): int(v) for k, v in zip(*np.unique(g, return_counts=True))}
    assert set(counts) == {-1, 0, 1, 2, 3, 4, 5, 6, 7}
    # inlet / main exit: the main vessel's cross-section interior on x = 3 / x = 272
    assert np.all(np.nonzero(g == 2)[2] == 3) and np.all(np.nonzero(g == 3)[2] == 272)
    assert counts[2] == counts[3]
    for code, z in ((5, 185), (6, 191), (7, 204)):
        assert np.all(np.nonzero(g == code)[0] == z)
    n_lattice, _ = lbm.index_transform(g)
    assert n_lattice == sum(v for k, v in counts.items() if k != 0)


def test_read_geo_txt_zxy(lbm, oracle, tmp_path):
    rng = np.random.default_rng(3)
    nz, ny, nx = 5, 4, 3
    raw = rng.integers(0, 2, (nz, ny, nx)).astype(np.int32)
    p = tmp_path / "geo.txt"
    # coronary.cu:45-56 reads z outer, then x, then y
    p.write_text(" ".join(str(int(raw[z, y, x])) for z in range(nz) for x in range(nx) for y in range(ny)))
    got = lbm.read_geo_txt_zxy(str(p), (nz, ny, nx))
    assert np.array_equal(got, raw)
    assert np.array_equal(oracle.read_geo_txt_zxy(str(p), nx, ny, nz), raw)
    with pytest.raises(lbm.LbmError):
        lbm.read_geo_txt_zxy(str(p), (nz + 1, ny, nx))


def test_coronary_initial_fields(lbm):
    from lbm_amd import cases
    raw, ends = cases.coronary_small_vessel()
    g = lbm.geo_ends(raw, ends)
    rho, ux, uy, uz = lbm.initial_fields(3, g)
    cu = f32(cases.CORONARY_C_U)
    # coronary.cu:298-307: float quotients
    want_ux = np.where(g == 2, f32(0.1745) / cu, np.where(g == 3, f32(0.1) / cu, f32(0))).astype(np.float32)
    want_uz = np.where((g >= 5) & (g <= 7), f32(0.02) / cu, f32(0)).astype(np.float32)
    assert np.array_equal(ux, want_ux) and np.array_equal(uz, want_uz)
    assert np.all(uy == 0) and np.all(rho == 1)


def vtk_coronary_expected(geo, rho, ux, uy, uz, C_U=2.74909090909091, CH=6.1111e-05, C_rho=1060.0):
    """coronary.cu:948-1011 written from the reference text (not lbmh_write_vtk): C++ ostream
    default formatting (%g, 6 significant digits); DENSITY rho*C_rho and VELOCITY u*C_U in
    float, PRESSURE rho*C_pre (float) / 3.0 in double; unstored cells print 0."""
    nz, ny, nx = geo.shape
    cu, ch, cr = f32(C_U), f32(CH), f32(C_rho)
    c_pre = cr * cu * cu
    head = ["# vtk DataFile Version 2.0",
            "<-- LBM flow with UIV acceleration, http://www.bg.ic.ac.uk/research/m.tang/ulis/ -->",
            "ASCII", "DATASET STRUCTURED_POINTS",
            f"DIMENSIONS {nx - 2} {ny - 4} {nz - 2}",
            "SPACING {0:g} {0:g} {0:g}".format(float(ch)),
            "ORIGIN {:g} {:g} {:g}".format(float(nx // 2) * float(ch), float(ny // 2) * float(ch), 0.0),
            f"POINT_DATA  {(nx - 2) * (ny - 4) * (nz - 2)}"]
    sl = (slice(1, nz - 1), slice(2, ny - 2), slice(1, nx - 1))
    st = geo[sl] != 0
    dens = np.where(st, (rho[sl] * cr).astype(np.float32), f32(0)).astype(np.float64)
    pres = np.where(st, (rho[sl] * c_pre).astype(np.float32).astype(np.float64) / 3.0, 0.0)
    vel = np.stack([np.where(st, (a[sl] * cu).astype(np.float32), f32(0)) for a in (ux, uy, uz)], -1)
    text = "\n".join(head) + "\n"
    text += "SCALARS DENSITY float\nLOOKUP_TABLE default\n" + "".join("%g " % v for v in dens.reshape(-1)) + "\n"
    text += "SCALARS PRESSURE float\nLOOKUP_TABLE default\n" + "".join("%g " % v for v in pres.reshape(-1)) + "\n"
    text += "VECTORS VELOCITY float\n" + "".join("%g " % v for v in vel.reshape(-1).astype(np.float64))
    return text


def test_coronary_vtk_format(lbm, tmp_path):
    from lbm_amd import cases
    raw, ends = cases.coronary_small_vessel()
    g = lbm.geo_ends(raw, ends)
    rng = np.random.default_rng(5)
    rho = (1 + rng.normal(0, 1e-3, g.shape)).astype(np.float32)
    ux, uy, uz = (rng.normal(0, 0.02, g.shape).astype(np.float32) for _ in range(3))
    p = tmp_path / "c.vtk"
    lbm.write_vtk_coronary(str(p), g, rho, ux, uy, uz)
    assert p.read_text() == vtk_coronary_expected(g, rho, ux, uy, uz)
