"""Two time steps per launch (k_step2: LDS temporal blocking) against the oracle, bit for bit.

LBM_TUNE_STEPS_PER_LAUNCH = 2 selects the two-step kernel (opt-in; one step per launch is the
default), wherever rows are a multiple of 64 slots, so small lattices exercise every boundary kind:
LDC walls + lid NEE (the racy-swap semantics, bounce-back already at step 0), Poiseuille inlet
/ outlet velocity NEE, the bifurcation's pressure outlet, both row axes, odd step counts (the
last step then runs on the one-step kernel) and the raw NEE pulls of step 0."""
import numpy as np
import pytest

from test_gpu_parity import assert_bitwise, assert_residuals

pytestmark = pytest.mark.gpu


@pytest.fixture
def two_steps(knob, lbm):
    knob(lbm.TUNE_STEPS_PER_LAUNCH, 2)


@pytest.mark.parametrize("n,steps", [(64, [2, 1, 4, 41]), (128, [2, 6])])
def test_ldc_two_step(gpu, oracle, two_steps, row_axis, n, steps):
    from lbm_amd import cases
    lat, geo = cases.ldc(n)
    o = oracle.Oracle(oracle.LDC, geo, 0.55, ldc_order=oracle.TWO_PHASE)
    for s in steps:
        hg, ho = lat.step(s), o.step(s)
        assert_bitwise(lat, o, geo, 0, f"ldc{n} +{s}")
        assert_residuals(hg, ho)
    assert lat.stats()["two_step_launches"] > 0


@pytest.mark.parametrize("shape", [(64, 64, 24), (128, 64, 20)])
def test_poiseuille_two_step(gpu, oracle, two_steps, row_axis, shape):
    from lbm_amd import cases
    nx, ny, nz = shape
    lat, geo = cases.poiseuille(nx, ny, nz)
    o = oracle.Oracle(oracle.POISEUILLE, geo, 0.58)
    for s in (2, 3, 30):
        hg, ho = lat.step(s), o.step(s)
        assert_bitwise(lat, o, geo, 1, f"poiseuille{shape} +{s}")
        assert_residuals(hg, ho)


@pytest.mark.parametrize("block", [0, 1])
def test_bifurcation_two_step(gpu, oracle, two_steps, knob, block):
    from lbm_amd import cases
    knob(gpu.TUNE_ROW_AXIS, 1)  # rows along x (64 slots); 83-cell y rows are not a multiple of 64
    lat, geo, inl, outl = cases.bifurcation(block)
    o = oracle.Oracle(oracle.MASK, geo, 0.55, inlet_uy=inl, outlet_uy=outl)
    for s in (2, 1, 60):
        hg, ho = lat.step(s), o.step(s)
        assert_bitwise(lat, o, geo, 2, f"bif{block} +{s}")
        # block 0 starts at rest behind a blocked inlet: 0/0 residuals on both sides
        np.testing.assert_allclose(hg, ho, rtol=0, atol=2e-4, equal_nan=block == 0)


def test_ldc256_two_step_matches_one_step(gpu, knob):
    """Two-step kernel at 256^3: field digests and residuals equal the one-step kernel's after
    an even and an odd number of steps."""
    from lbm_amd import cases
    import lbm_amd
    a = cases.ldc_device(256, 256, 256)
    knob(lbm_amd.TUNE_STEPS_PER_LAUNCH, 1)
    b = cases.ldc_device(256, 256, 256)
    for s in (10, 5):
        knob(lbm_amd.TUNE_STEPS_PER_LAUNCH, 2)
        ha = a.step(s)
        knob(lbm_amd.TUNE_STEPS_PER_LAUNCH, 1)
        hb = b.step(s)
        np.testing.assert_allclose(ha, hb, rtol=0, atol=1e-7)  # fp64 partial sums in another order
        assert np.array_equal(a.digest(), b.digest())
    assert a.stats()["two_step_launches"] >= 5 and b.stats()["two_step_launches"] == 0
