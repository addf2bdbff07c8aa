"""coronary_cfd/coronary.cu on the GPU: its geo_pre (lbmh_geo_ends) + boundary
codes (LBM_CASE_GENERIC, cases.coronary_bc_codes) + initialize() stepped by liblbm, bit for bit
against the oracle (orc_geo_coronary, the generic NEE restatement of coronary.cu:716-943 and
orc_initialize_coronary), and the drop-in driver bin/coronary (coronary.cu main 1055-1163) with
its VTK snapshots and CONVERGENCE.log against the oracle's fields rendered by the independent
writer of tests/test_coronary.py.  The reference's geo.txt is not shipped: synthetic vessel
trees whose open ends sit on coronary.cu's end planes stand in for it."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG
from test_coronary import vtk_coronary_expected
from test_gpu_parity import assert_bitwise, assert_residuals

pytestmark = pytest.mark.gpu


def _oracle(oracle, geo):
    from lbm_amd import cases
    o = oracle.Oracle(oracle.GENERIC, geo, cases.CORONARY_TAU, bcs=cases.coronary_bc_codes())
    o.initialize_coronary()
    o.residual_fp64(True)  # liblbm's summation (assert_residuals)
    return o


def test_coronary_small_vessel_bitwise(gpu, oracle, cells_per_lane, row_axis):
    from lbm_amd import cases
    raw, ends = cases.coronary_small_vessel()
    lat, geo = cases.coronary(raw, ends)
    assert np.array_equal(geo, oracle.geo_coronary(raw, ends))
    o = _oracle(oracle, geo)
    assert np.array_equal(lat.f()[:, geo != 0].view(np.uint32), o.f()[:, geo != 0].view(np.uint32))
    for s in (1, 1, 60):
        hg, ho = lat.step(s), o.step(s)
        assert_bitwise(lat, o, geo, 2, f"coronary small +{s}")
        assert_residuals(hg, ho)
    assert o.bad_reads() == 0
    lat.close()


def test_coronary_reference_box_bitwise(gpu, oracle):
    """The reference's 291 x 291 x 372 box with its own five end planes (coronary.cu:75-143)."""
    from lbm_amd import cases
    raw = cases.coronary_reference_vessel()
    lat, geo = cases.coronary(raw)
    o = _oracle(oracle, geo)
    for s in (1, 2):
        hg, ho = lat.step(s), o.step(s)
        assert_bitwise(lat, o, geo, 2, f"coronary 291x291x372 +{s}")
        assert_residuals(hg, ho)
    lat.close()


def _calc_res_fluid(geo, ux, uy, uz):
    """coronary.cu:1013-1031: fp32 |u|^2 over code 4 in the output region, long double, z, y, x."""
    sl = (slice(1, geo.shape[0] - 1), slice(2, geo.shape[1] - 2), slice(1, geo.shape[2] - 1))
    m = geo[sl] == 4
    v = (ux[sl] * ux[sl] + uy[sl] * uy[sl]) + uz[sl] * uz[sl]
    terms = v[m].astype(np.longdouble)
    return np.cumsum(terms)[-1] if terms.size else np.longdouble(0)


def test_coronary_driver(gpu, oracle, tmp_path):
    """bin/coronary on a small vessel (--nx/--ny/--nz and its own --ends table): snapshots at
    i % time_save == 0 byte for byte, CONVERGENCE.log residuals and the stdout lines."""
    from lbm_amd import cases
    from test_gpu_drivers import _cfmt
    raw, ends = cases.coronary_small_vessel()
    nz, ny, nx = raw.shape
    # geo.txt in coronary.cu's z, x, y order
    (tmp_path / "geo.txt").write_text(" ".join(map(str, raw.transpose(0, 2, 1).reshape(-1).tolist())))
    table = ";".join(",".join(map(str, e)) for e in ends)
    r = subprocess.run([os.path.join(PKG, "bin", "coronary"), "--nx", str(nx), "--ny", str(ny), "--nz", str(nz),
                        "--ends", table, "--repeat", "40", "--time-save", "20", "--out", "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300, check=True)
    lines = r.stdout.strip().splitlines()
    assert [x.split(",")[0] for x in lines[:3]] == ["ITERATION # 0", "ITERATION # 20", "ITERATION # 40"]
    geo = oracle.geo_coronary(raw, ends)
    n_lattice, _ = oracle.index_transform(geo)
    assert re.fullmatch(rf"TOTAL RUNNING TIME: [0-9.e+-]+ MILLI SECONDS#LATTICE{n_lattice}", lines[-1])
    o = _oracle(oracle, geo)
    # host arrays before the first copy-back: initialize()'s fields (coronary.cu:298-307)
    cu = np.float32(cases.CORONARY_C_U)
    prev = (np.where(geo == 2, np.float32(0.1745) / cu, np.where(geo == 3, np.float32(0.1) / cu, 0)).astype(np.float32),
            np.zeros(geo.shape, np.float32),
            np.where((geo >= 5) & (geo <= 7), np.float32(0.02) / cu, 0).astype(np.float32))
    residuals = []
    done = 0
    for k in (0, 20, 40):
        o.step(k + 1 - done)
        done = k + 1
        rho, ux, uy, uz = o.macros()
        got = (tmp_path / "out" / f"coronary_{k}.vtk").read_text()
        assert got == vtk_coronary_expected(geo, rho, ux, uy, uz), f"coronary_{k}.vtk"
        s1, s2 = _calc_res_fluid(geo, *prev), _calc_res_fluid(geo, ux, uy, uz)
        residuals.append(np.float32(abs(s1 - s2) / s2))
        prev = (ux, uy, uz)
    log = (tmp_path / "out" / "CONVERGENCE.log").read_text().strip().splitlines()
    assert log[:3] == [_cfmt(v) for v in residuals]
    assert log[3].endswith(" ERROR IS" + _cfmt(residuals[-1]))
