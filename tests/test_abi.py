"""The C-ABI boundary (include/*.h): every declared function is exported by the built
library and bound by the Python mirror; the libraries load on a CPU-only host and fail
loudly (no CPU fallback) where a device is needed.  No compute runs here."""
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO

HEADERS = {
    "lbm.h": os.path.join(PKG, "lib", "liblbm.so"),
    "lbm_host.h": os.path.join(PKG, "lib", "liblbm_host.so"),
}
DECL = re.compile(r"^\s*(?:const\s+)?(?:long\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*\b(lbmh?_[a-z0-9_]+)\s*\(", re.M)


def declared(header: str):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(DECL.findall(text)))


def exported(lib: str):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


@pytest.mark.parametrize("header", sorted(HEADERS))
def test_header_symbols_exported(header):
    names = declared(header)
    assert len(names) >= 10
    lib = HEADERS[header]
    assert os.path.exists(lib), f"{lib} not built (make -C {PKG})"
    missing = set(names) - exported(lib)
    assert not missing, f"{os.path.basename(lib)} lacks {sorted(missing)}"


def test_python_mirror_binds_every_symbol(lbm):
    assert sorted(lbm.LBM_SYMBOLS) == declared("lbm.h")
    assert sorted(lbm.HOST_SYMBOLS) == declared("lbm_host.h")
    L, H = lbm.lbm_lib(), lbm.host_lib()
    for name in lbm.LBM_SYMBOLS:
        assert getattr(L, name).argtypes is not None, name
    for name in lbm.HOST_SYMBOLS:
        assert getattr(H, name).argtypes is not None, name


@pytest.mark.parametrize("name", ["lbm_desc", "lbm_bc_code"])
def test_struct_layout_matches_header(lbm, name):
    """Field order of the ctypes mirrors follows include/lbm.h."""
    text = open(os.path.join(REPO, "include", "lbm.h")).read()
    end = text.index("} " + name + ";")
    body = text[text.rindex("typedef struct {", 0, end):end]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"\b([a-z_][a-z0-9_]*)\s*(?:\[\d+\])?\s*(?:,|;)", body)
    assert [f[0] for f in getattr(lbm, name)._fields_] == fields


def test_loads_without_device_and_fails_loudly(lbm):
    """Version works with no GPU; creating a context without a device is an error with a
    message -- never a silent CPU fallback."""
    assert "gfx950" in lbm.version()
    if lbm.gpu_available():
        pytest.skip("a device is visible")
    with pytest.raises(lbm.LbmError, match="hipSetDevice|device"):
        lbm.Lattice(lbm.LBM_CASE_LDC, (8, 8, 8), 0.55, None)
    with pytest.raises(lbm.LbmError):
        lbm.require_gpu()


def test_invalid_descriptions_rejected(lbm):
    with pytest.raises(lbm.LbmError, match="invalid lattice description"):
        lbm.Lattice(lbm.LBM_CASE_LDC, (8, 8, 2), 0.55, None)  # nx < 3
    with pytest.raises(lbm.LbmError, match="invalid lattice description"):
        lbm.Lattice(lbm.LBM_CASE_LDC, (8, 8, 8), -1.0, None)
    with pytest.raises(lbm.LbmError, match="geo == NULL"):
        lbm.Lattice(lbm.LBM_CASE_POISEUILLE, (8, 8, 8), 0.58, None)
    with pytest.raises(lbm.LbmError, match="invalid lattice description"):
        lbm.Lattice(lbm.LBM_CASE_LDC, (8, 8, 8), 0.55, None, x_align=7)
    # device mask build: MASK case only, ny >= 5, slabs need halo planes
    import numpy as np
    with pytest.raises(lbm.LbmError, match="geo == NULL"):
        lbm.Lattice(lbm.LBM_CASE_POISEUILLE, (8, 8, 8), 0.58, None, mask=np.ones((8, 8, 8), np.uint8))
    with pytest.raises(lbm.LbmError, match="ny >= 5"):
        lbm.Lattice(lbm.LBM_CASE_MASK, (8, 4, 8), 0.55, None, mask=np.ones((8, 4, 8), np.uint8))
    with pytest.raises(lbm.LbmError, match="halo_planes"):
        lbm.Lattice(lbm.LBM_CASE_MASK, (8, 8, 8), 0.55, None, mask=np.ones((8, 8, 8), np.uint8), z_offset=8,
                    nz_global=16)
    with pytest.raises(lbm.LbmError, match="mask shape"):
        lbm.Lattice(lbm.LBM_CASE_MASK, (8, 8, 8), 0.55, None, mask=np.ones((8, 8, 8), np.uint8), halo_planes=True)


def test_tune_knobs_validated(lbm):
    """lbm_tune (host only, no device needed): returns the previous value, rejects unknown
    knobs and out-of-range values with LBM_ERR_ARG, and the defaults are the documented ones."""
    defaults = {lbm.TUNE_ROW_AXIS: 0, lbm.TUNE_CELLS_PER_LANE: 0, lbm.TUNE_EXACT_DIV: 0,
                lbm.TUNE_FUSED_RESIDUAL: 1, lbm.TUNE_BUFFER_ALLOC: 0, lbm.TUNE_SYNC_TIMEOUT_S: 0,
                lbm.TUNE_GRID_STRIDE: 0, lbm.TUNE_INJECT_RCCL_FAULT: 0, lbm.TUNE_GROUPS: 0,
                lbm.TUNE_GROUP_SEGMENT: 16, lbm.TUNE_COMPACT: 0, lbm.TUNE_BOX: 0, lbm.TUNE_NEE_FIX: 0,
                lbm.TUNE_XCD_RUN: 0, lbm.TUNE_NEE_ORDER: 0}
    for knob, dflt in defaults.items():
        assert lbm.tune(knob, dflt) == dflt
    with lbm.tuned(lbm.TUNE_CELLS_PER_LANE, 4):
        assert lbm.tune(lbm.TUNE_CELLS_PER_LANE, 4) == 4
    assert lbm.tune(lbm.TUNE_CELLS_PER_LANE, 0) == 0
    for knob, value in ((-1, 0), (len(defaults), 0), (lbm.TUNE_ROW_AXIS, 3), (lbm.TUNE_CELLS_PER_LANE, 2),
                        (lbm.TUNE_CELLS_PER_LANE, 3), (lbm.TUNE_EXACT_DIV, -1), (lbm.TUNE_SYNC_TIMEOUT_S, 86401),
                        (lbm.TUNE_GRID_STRIDE, 9), (lbm.TUNE_INJECT_RCCL_FAULT, 1), (lbm.TUNE_GROUPS, 3),
                        (lbm.TUNE_GROUP_SEGMENT, 65), (lbm.TUNE_COMPACT, 3), (lbm.TUNE_BOX, 2),
                        (lbm.TUNE_NEE_FIX, 4), (lbm.TUNE_XCD_RUN, 18), (lbm.TUNE_BUFFER_ALLOC, 3),
                        (lbm.TUNE_NEE_ORDER, 3)):
        with pytest.raises(lbm.LbmError, match="unknown knob or value"):
            lbm.tune(knob, value)
    for knob, dflt in defaults.items():  # a rejected call leaves every knob as it was
        assert lbm.tune(knob, dflt) == dflt


def test_drivers_built():
    for exe in ("ldc", "poiseuille", "bifurcation"):
        assert os.access(os.path.join(PKG, "bin", exe), os.X_OK), exe
