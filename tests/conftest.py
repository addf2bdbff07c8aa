"""Test configuration: `gpu` marks tests that need an MI355X (run with -m gpu on the GPU
box); everything else runs on the CPU container.  The oracle (oracle/) is the checker."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "lattice-boltzmann-method-gpu_amd")
for p in (REPO, PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long CPU-only oracle runs (excluded by default selection)")


@pytest.fixture(scope="session")
def oracle():
    import orc
    orc.build()
    return orc


@pytest.fixture(scope="session")
def lbm():
    import lbm_amd
    return lbm_amd


@pytest.fixture(scope="session")
def gpu(lbm):
    lbm.require_gpu()
    return lbm


@pytest.fixture
def knob(lbm):
    """knob(which, value): set an lbm_tune knob for the rest of the test (restored after)."""
    saved = []

    def set_(which, value):
        saved.append((which, lbm.tune(which, value)))

    yield set_
    for which, prev in reversed(saved):
        lbm.tune(which, prev)


@pytest.fixture(params=["4", "4g", "4c", "1", "1g", "1c"],
                ids=["4cells", "4groups", "4compact", "1cell", "1groups", "1compact"])
def cells_per_lane(request, knob, lbm):
    """Run a parity test through every stream-collide path: four cells per lane over whole
    chunks (the bandwidth path), four cells per lane over compact lists of active 4-cell groups
    (sparse lattices; forced on every sparse chunk list) in the dense box and in compact rows
    (LBM_TUNE_COMPACT 2: single-domain lattices whose list is sparse), one cell per lane over whole
    chunks (what small lattices use by default) and one cell per lane over the group lists, dense
    and compact."""
    knob(lbm.TUNE_CELLS_PER_LANE, 4 if request.param.startswith("4") else 1)
    knob(lbm.TUNE_GROUPS, 1 if len(request.param) == 1 else 2)
    knob(lbm.TUNE_COMPACT, 2 if request.param.endswith("c") else 1)
    return 4 if request.param.startswith("4") else 1


@pytest.fixture(params=["x", "y"], ids=["xrows", "yrows"])
def row_axis(request, knob, lbm):
    """Run a parity test on both device layouts: rows along x and rows along y
    (lbm_desc.row_axis; LBM_TUNE_ROW_AXIS stands in for row_axis = 0)."""
    knob(lbm.TUNE_ROW_AXIS, 1 if request.param == "x" else 2)
    return request.param
