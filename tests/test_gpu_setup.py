"""What lbm_create costs (lbm_get_setup_cost) and where the NEE values of a step come from
(lbm_get_nee_path): the device memory a context holds against its population buffers, the
transient peak of the buffer-placement probe, and the compact (rho, u) records of k_nee_fix."""
import pytest

pytestmark = pytest.mark.gpu

# device bytes per cell slot besides the populations: type byte, reference code, wall-link and
# NEE-link masks, and the four macro floats (the NEE cells' boundary data, lazy read-outs)
PER_CELL = 1 + 1 + 4 + 4 + 16


def test_pipe_device_bytes(gpu):
    """C3's pipe (128 x 512 x 128, rows along y) with k_nee_fix (LBM_TUNE_NEE_FIX 3), whose (rho, u) records are one
    16-B slot per NEE-adjacent cell (25.7 k cells), not one per box cell (8.4 M: 134 MB more,
    round 5).  The context holds its two population buffers plus 26 B per cell slot and small
    work lists; the placement probe's candidates are gone when lbm_create returns."""
    from lbm_amd import cases
    import lbm_amd
    with lbm_amd.tuned(lbm_amd.TUNE_NEE_FIX, 3):
        lat, _ = cases.poiseuille(128, 512, 128)
    assert lat.nee_path()["path"] == "fix"
    st, sc = lat.storage(), lat.setup_cost()
    expect = st["bytes"] + PER_CELL * st["cells"]
    print("C3 setup", sc, "expected ~", expect)
    assert st["bytes"] <= sc["device_bytes"] <= expect * 1.02 + (64 << 20), (sc, expect)
    assert sc["device_bytes"] <= sc["peak_bytes"] <= sc["device_bytes"] + (160 << 30)
    assert sc["create_s"] > 0
    lat.close()


def test_placement_peak_is_reported(gpu):
    """LDC 256^3 (1.28-GB buffers, over the 256-MB threshold): lbm_create holds up to 64
    placement candidates at once; the peak it reports covers them, and the memory it keeps is
    the two chosen buffers plus the per-cell arrays."""
    from lbm_amd import cases
    lat = cases.ldc_device(256, 256, 256)
    st, sc, pl = lat.storage(), lat.setup_cost(), lat.placement()
    n = len(pl["candidate_write_gbs"])
    assert 2 <= n <= 64
    one = st["bytes"] // 2
    assert sc["peak_bytes"] >= n * one * 0.99, (sc, n, one)
    assert sc["device_bytes"] <= st["bytes"] + PER_CELL * st["cells"] + (64 << 20), sc
    lat.close()


@pytest.mark.parametrize("case", ["pipe", "bif_x4"])
def test_nee_fix_records_compact(gpu, knob, case):
    """k_nee_fix's records numbered by storage rank: the pipe's chunk list (one NEE-adjacent cell
    per chunk) and the upsampled bifurcation's compact 4-cell group list (64-entry slices, several
    NEE-adjacent cells per wave; LBM_TUNE_NEE_FIX 3) against the default NEE path (NEE blocks),
    bit for bit -- which the oracle pins (test_poiseuille_nee_paths_bitwise,
    test_bifurcation_upsampled_bitwise)."""
    import numpy as np
    from lbm_amd import cases
    import lbm_amd
    knob(lbm_amd.TUNE_CELLS_PER_LANE, 4)

    def run(mode):
        with lbm_amd.tuned(lbm_amd.TUNE_NEE_FIX, mode):
            lat = cases.poiseuille(44, 300, 40)[0] if case == "pipe" else cases.bifurcation_upsampled(4)[0]
        path = lat.nee_path()["path"]
        h = lat.step(13)
        fluid = lat.geo() == 4
        f = lat.f()[:, fluid]
        m = np.stack(lat.macros())[:, fluid]
        lat.close()
        return path, h, f, m

    p0, h0, f0, m0 = run(3)
    p1, h1, f1, m1 = run(0)
    assert (p0, p1) == ("fix", "blocks")
    assert np.array_equal(f0.view(np.uint32), f1.view(np.uint32))
    assert np.array_equal(m0.view(np.uint32), m1.view(np.uint32))
    assert np.allclose(h0, h1, rtol=0, atol=2e-7)
