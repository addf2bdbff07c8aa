"""BASELINE configs end to end on the GPU, and the loop semantics around the hot path.

* C5 (LDC 512 x 512 x 4096, ldc.cu:468-502 at the 8-GPU size) on ONE GPU: the whole lattice
  as one domain (1.07 G cells, ~187 GB of HBM), then the same lattice as 8 z-slabs of 512^3
  stepped together with the halo exchange (lbm_group_step, device-to-device copies standing in
  for RCCL).  The per-plane field digests (lbm_field_digest: keyed by global coordinates, so
  independent of the cut) must agree plane for plane: the decomposition is exercised at C5's
  exact shape and halo size.
* C1 and the Poiseuille default loop to convergence (ldc.cu:653-691, Poiseulle.cu:986-1030):
  stop step and field bits against the oracle run recorded in tests/golden/converge.json
  (tests/golden/make_converge.py).
* the NaN guard of the residual (not in the reference).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_c5_single_gpu_vs_8_slabs(gpu):
    from lbm_amd import cases
    import lbm_amd
    n, nzg, steps = 512, 4096, 5
    one = cases.ldc_device(n, n, nzg)
    c = one.counts()
    assert c["n_box"] == n * n * nzg and c["n_fluid"] == (n - 4) ** 2 * (nzg - 4)
    h1 = one.step(steps)
    assert np.all(np.isfinite(h1))
    d_one = one.digest()
    st = one.state()
    one.close()
    del one
    assert st["k"] == steps
    slabs = [cases.ldc_device(n, n, n, z_offset=i * n, nz_global=nzg) for i in range(8)]
    hs = lbm_amd.group_step(slabs, steps)
    # the same |u| sums up to fp64 summation order: identical fp32 residuals
    np.testing.assert_allclose(hs, h1, rtol=0, atol=1e-7)
    for i, lat in enumerate(slabs):
        d = lat.digest()
        bad = np.nonzero(d != d_one[i * n:(i + 1) * n])[0]
        assert bad.size == 0, f"slab {i}: planes {bad[:8] + i * n} differ from the single-domain run"
        lat.close()


def _converge(name):
    return json.load(open(os.path.join(GOLDEN, "converge.json")))[name]


def _sha_fluid(macros, fluid):
    import hashlib
    h = hashlib.sha256()
    for a in macros:
        h.update(np.ascontiguousarray(a[fluid]).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("name", ["ldc64_two_phase", "poiseuille64"])
def test_default_loop_converges_like_oracle(gpu, name):
    """The reference's own default loop to convergence on the GPU: the same stop step as the
    oracle with the same (fp64-accumulated) |u| sum, and the same field bits there.  The
    survey's emulation of thrust's fp32 sum (serial, storage order) stops elsewhere -- that
    difference is the summation order alone."""
    from lbm_amd import cases
    g = _converge(name)
    if name.startswith("ldc"):
        lat, geo = cases.ldc(64)
        fluid = geo == 3
    else:
        lat, geo = cases.poiseuille(64, 64, 64)
        fluid = geo == 4
    lat.set_convergence(True, 10000, 50, 1e-6)
    lat.step(10001, history=False)
    st = lat.state()
    assert st["stopped"] == 1 and st["nonfinite_k"] == 0
    assert st["k"] == g["stop_k_fp64"], (st["k"], g)
    assert np.float32(st["residual"]) == np.float32(g["residual_fp64"])
    assert _sha_fluid(lat.macros(), fluid) == g["sha256_macros_fluid_fp64_stop"]
    if name == "poiseuille64":
        # reference-held (thesis, oracle/PINNING.md section 1): "~6200" steps to convergence
        # (Table 4-3) and < 2 % error against the analytical solution (section 4.9.2), here the
        # centre-line velocity against the imposed parabola's peak (Poiseulle.cu:590)
        assert abs(st["k"] - 6200) <= 0.03 * 6200
        uy = lat.macros()[2]
        umax = float(uy[fluid].max())
        assert abs(umax - 0.09714700668) / 0.09714700668 < 0.02, umax
    lat.close()


@pytest.mark.parametrize("name,params", [("ldc64_two_phase", "cub_i16_v4_g240"), ("poiseuille64", "thrust_i20_v2_g240")])
def test_reference_order_residual_stop_step(gpu, name, params):
    """lbm_set_residual_order(LBM_SUM_CUB_TREE): the |u| terms in the reference's storage order
    summed in fp32 by thrust::reduce's CUB tree.  The default loop stops at exactly the oracle's
    step under the same tree (tests/golden/residual_order.json, make_residual_order.py), with
    the same last residual and field bits there -- 5084 / 6334, against 5080 / 6333 with the
    default fp64 sum and 5711 / 6230 with a serial fp32 sum."""
    import lbm_amd
    from lbm_amd import cases
    g = json.load(open(os.path.join(GOLDEN, "residual_order.json")))[name][params]
    if name.startswith("ldc"):
        lat, geo = cases.ldc(64)
        fluid = geo == 3
    else:
        lat, geo = cases.poiseuille(64, 64, 64)
        fluid = geo == 4
    lat.set_residual_order(lbm_amd.LBM_SUM_CUB_TREE, *g["params_ipt_vec_grid"])
    lat.set_convergence(True, 10000, 50, 1e-6)
    lat.step(10001, history=False)
    st = lat.state()
    assert st["stopped"] == 1 and st["k"] == g["stop_k"], (st["k"], g["stop_k"])
    assert np.float32(st["residual"]) == np.float32(g["residual"])
    assert _sha_fluid(lat.macros(), fluid) == g["sha256_macros_fluid_stop"]
    lat.close()


@pytest.mark.parametrize("case", ["ldc_ragged", "bifurcation"])
def test_reference_order_residual_history(gpu, case):
    """The CUB-tree residual history step by step against the oracle's, bit for bit: the LDC
    brick order on a box that is not a multiple of the 8-cell bricks, and index_transform's
    compact order on the shipped bifurcation (several tiles per block: grid_cap 3)."""
    import lbm_amd
    import orc
    from lbm_amd import cases
    if case == "ldc_ragged":
        lat, geo = cases.ldc(36, 27, 21)
        o = orc.Oracle(orc.LDC, geo, 0.55, ldc_order=orc.TWO_PHASE)
        params = (16, 4, 240)
    else:
        lat, geo, inl, outl = cases.bifurcation(1)
        o = orc.Oracle(orc.MASK, geo, 0.55, inlet_uy=inl, outlet_uy=outl)
        params = (20, 2, 3)
    lat.set_residual_order(lbm_amd.LBM_SUM_CUB_TREE, *params)
    o.residual_cub_tree(*params)
    h = lat.step(60)
    oh = o.step(60)
    assert np.array_equal(np.asarray(h, np.float32).view(np.uint32), np.asarray(oh, np.float32).view(np.uint32))
    lat.close()


def test_drivers_default_loop_stop_step(gpu, tmp_path):
    """bin/ldc and bin/poiseuille with no size arguments (the reference's 64^3 mains, C1):
    snapshots every 500 steps, then the final snapshot named by the pinned stop step, and the
    last residual printed as the reference prints it (ldc.cu:686-697)."""
    import subprocess
    from conftest import PKG
    for exe, name, prefix in (("ldc", "ldc64_two_phase", "lid"), ("poiseuille", "poiseuille64", "pos")):
        g = _converge(name)
        k = g["stop_k_fp64"]
        out = tmp_path / exe
        r = subprocess.run([os.path.join(PKG, "bin", exe), "--out", str(out)], capture_output=True, text=True,
                           timeout=300, check=True)
        lines = r.stdout.strip().splitlines()
        its = [int(x.split("# ")[1].split(",")[0]) for x in lines if x.startswith("ITERATION")]
        assert its == list(range(0, k, 500)), (its[-3:], k)
        assert lines[-1] == "Residual is %g" % np.float32(g["residual_fp64"])
        assert os.path.exists(out / f"{prefix}_{k}.vtk"), sorted(os.listdir(out))[-3:]


def test_nan_guard(gpu, oracle):
    """A NaN population makes the step's |u| sum non-finite: recorded (lbm_get_nonfinite) with
    or without convergence control, and under convergence control the run stops (stopped 2)."""
    from lbm_amd import cases
    for conv in (False, True):
        lat, geo = cases.ldc(16)
        f = lat.f()
        f[3, 8, 8, 8] = np.nan
        lat.set_f(f)
        if conv:
            lat.set_convergence(True, 10000, 50, 1e-6)
        lat.step(20, history=False)
        st = lat.state()
        assert st["nonfinite_k"] == 1
        if conv:
            assert st["stopped"] == 2 and st["k"] == 1
        else:
            assert st["k"] == 20
        lat.close()


def test_probe_stream_shapes(gpu):
    """lbm_probe_stream_shapes: a rate for every copy shape (register and LDS-DMA tiles
    included), and lbm_probe_stream reports their best."""
    import lbm_amd
    per = lbm_amd.probe_stream_shapes(0, 256 << 20, 2)
    assert list(per) == lbm_amd.PROBE_SHAPES, per
    assert all(v > 0 for v in per.values()), per
    best = lbm_amd.probe_stream(0, 256 << 20, 2)
    assert 0.5 * max(per.values()) < best < 2.0 * max(per.values())
