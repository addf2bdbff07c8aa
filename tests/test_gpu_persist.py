"""The persistent multi-step path (k_persist: one launch per lbm_step call, workgroups waiting
on the workgroups they pull from instead of a launch boundary per step) against the
one-launch-per-step path (k_step1) on the same lattices: populations, macros and the NEE
cells' kept (rho, u) bit for bit after every call, convergence stops at the same step."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(knob, lbm, make):
    knob(lbm.TUNE_CELLS_PER_LANE, 1)
    knob(lbm.TUNE_PERSISTENT, 1)
    ref = make()
    knob(lbm.TUNE_PERSISTENT, 0)
    per = make()
    assert ref.step_path()[0] == 1
    assert per.step_path()[0] == 2, per.step_path()
    return ref, per


def _same(a, b, what):
    for name, x, y in zip(("rho", "ux", "uy", "uz"), a.macros(), b.macros()):
        bad = np.count_nonzero(x.view(np.uint32) != y.view(np.uint32))
        assert bad == 0, f"{what} {name}: {bad} cells differ"
    fa, fb = a.f(), b.f()
    assert np.array_equal(fa.view(np.uint32), fb.view(np.uint32)), f"{what}: populations differ"


def test_default_paths(gpu):
    """Small single-domain lattices take the persistent path, large ones one launch per step."""
    from lbm_amd import cases
    assert cases.ldc_device(64, 64, 64).step_path()[0] == 2
    assert cases.ldc_device(128, 128, 128).step_path()[0] == 1
    lat, _, _, _ = cases.bifurcation(1)
    assert lat.step_path()[0] == 2


@pytest.mark.parametrize("case", ["ldc40", "ldc_ragged", "poiseuille", "bif0", "bif1", "generic", "coronary"])
def test_persist_equals_per_step(gpu, knob, case):
    from lbm_amd import cases
    import lbm_amd

    def make():
        if case == "ldc40":
            return cases.ldc(40)[0]
        if case == "ldc_ragged":
            return cases.ldc_device(37, 29, 23)
        if case == "poiseuille":
            return cases.poiseuille(32, 48, 40)[0]
        if case in ("bif0", "bif1"):
            return cases.bifurcation(int(case[-1]))[0]
        if case == "generic":
            return cases.generic(*cases.duct_generic(40, 22, 18), tau=0.6)
        raw, ends = cases.coronary_small_vessel()
        return cases.coronary(raw, ends)[0]

    ref, per = _pair(knob, lbm_amd, make)
    for n in (1, 2, 7, 30, 1, 61):
        hr = ref.step(n)
        hp = per.step(n)
        np.testing.assert_allclose(hp, hr, rtol=0, atol=1e-6)
        _same(ref, per, f"{case} +{n}")
    assert ref.state()["k"] == per.state()["k"]


def test_persist_no_history_calls(gpu, knob):
    """Calls without history or a steps_done read (asynchronous) keep the buffer parity."""
    from lbm_amd import cases
    import lbm_amd
    ref, per = _pair(knob, lbm_amd, lambda: cases.bifurcation(0)[0])
    for n in (3, 1, 1, 40, 5):
        ref.step(n, history=False)
        per.step(n, history=False)
    _same(ref, per, "bif async")


def test_persist_convergence_stop(gpu, knob):
    """Under convergence control the persistent launch runs at most one step past the stop
    step speculatively; the visible state is the stop step's, as in the per-step path."""
    from lbm_amd import cases
    import lbm_amd
    ref, per = _pair(knob, lbm_amd, lambda: cases.ldc(24)[0])
    for lat in (ref, per):
        lat.set_convergence(True, max_it=10000, stag_max=50, tol=1e-6)
    ks = []
    for lat in (ref, per):
        while True:
            lat.step(333)
            st = lat.state()
            if st["stopped"]:
                break
            assert st["k"] < 20000
        ks.append(st["k"])
    assert ks[0] == ks[1], ks
    _same(ref, per, f"ldc24 converged at {ks[0]}")
    per.step(7)
    assert per.state()["k"] == ks[1]
    _same(ref, per, "after no-op steps")


def test_persist_checkpoint_resume(gpu, knob, tmp_path):
    """The NEE cells' kept (rho, u) live in two arrays by step parity inside a launch; after
    the call the final ones are in the canonical list (what checkpoints save)."""
    from lbm_amd import cases
    import lbm_amd
    ref, per = _pair(knob, lbm_amd, lambda: cases.bifurcation(1)[0])
    ref.step(13)
    per.step(13)
    path = str(tmp_path / "p.ckpt")
    per.checkpoint_save(path)
    knob(lbm_amd.TUNE_PERSISTENT, 0)
    back = cases.bifurcation(1)[0]
    back.checkpoint_load(path)
    ref.step(20)
    back.step(20)
    _same(ref, back, "bif resumed")
