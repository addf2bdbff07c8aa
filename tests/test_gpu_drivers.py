"""The drop-in case drivers (lattice-boltzmann-method-gpu_amd/bin/*, the reference mains on
top of liblbm) against the oracle: same VTK snapshots, byte for byte, at the reference's
save steps (ldc.cu:653-691: a snapshot after step k+1 when k % time_save == 0, and one after
the loop), plus the stdout / CONVERGENCE.log line formats."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu
BIN = os.path.join(PKG, "bin")


def _oracle_vtk(lbm, oracle, geo, steps, path, kind, C_U, CH, **kw):
    o = oracle.Oracle(kind, geo, kw.pop("tau"), **kw)
    o.step(steps)
    rho, ux, uy, uz = o.macros()
    lbm.write_vtk(path, {oracle.LDC: 0, oracle.POISEUILLE: 1, oracle.MASK: 2}[kind], geo, ux, uy, uz, C_U, CH)
    return open(path).read()


def test_ldc_driver(gpu, oracle, tmp_path):
    n, max_it, save = 24, 25, 10
    out = tmp_path / "out"
    r = subprocess.run([os.path.join(BIN, "ldc"), "--nx", str(n), "--ny", str(n), "--nz", str(n), "--max-it",
                        str(max_it), "--time-save", str(save), "--out", str(out)],
                       capture_output=True, text=True, timeout=300, check=True)
    lines = r.stdout.strip().splitlines()
    assert re.fullmatch(r"ITERATION # 0, collapse time: [0-9.e+-]+ ms, residual:[0-9.e+-]+", lines[0])
    assert [int(re.search(r"# (\d+),", x).group(1)) for x in lines if x.startswith("ITERATION")] == [0, 10, 20]
    assert re.fullmatch(r"TOTAL RUNNING TIME: [0-9.e+-]+ MILLI SECONDS#LATTICE\d+", lines[-2])
    assert lines[-1].startswith("Residual is ")
    log = (out / "CONVERGENCE.log").read_text().strip().splitlines()
    assert len(log) == 4 and log[-1].startswith("TOTAL RUNNING TIME:") and " ERROR IS" in log[-1]
    geo = gpu.geo_ldc(n, n, n)
    C_U, CH = 2.4705, 0.0000655737
    for k, steps in ((0, 1), (10, 11), (20, 21), (max_it + 1, max_it + 1)):
        got = (out / f"lid_{k}.vtk").read_text()
        want = _oracle_vtk(gpu, oracle, geo, steps, str(tmp_path / f"o{k}.vtk"), oracle.LDC, C_U, CH, tau=0.55)
        assert got == want, f"lid_{k}.vtk differs from the oracle's"


def test_poiseuille_driver(gpu, oracle, tmp_path):
    nx, ny, nz = 20, 24, 20
    out = tmp_path / "out"
    subprocess.run([os.path.join(BIN, "poiseuille"), "--nx", str(nx), "--ny", str(ny), "--nz", str(nz),
                    "--max-it", "12", "--time-save", "6", "--out", str(out)],
                   capture_output=True, text=True, timeout=300, check=True)
    geo = gpu.geo_poiseuille(nx, ny, nz)
    files = sorted(os.listdir(out))
    assert "CONVERGENCE.log" in files
    got = (out / "pos_6.vtk").read_text()
    want = _oracle_vtk(gpu, oracle, geo, 7, str(tmp_path / "o.vtk"), oracle.POISEUILLE, 1.5441, 0.0000655737,
                       tau=0.58)
    assert got == want
