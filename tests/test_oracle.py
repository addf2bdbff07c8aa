"""The CPU oracle (oracle/, test infrastructure) against its pins and the golden vectors.

* pins.json holds full runs of oracle/pin_check.py against the known answers SURVEY.md
  records for the reference (oracle/PINNING.md); every recorded value must match.
* golden.json / golden.npz (tests/golden/make_golden.py) are re-derived here bit for bit.
* The long convergence pins re-run only with LBM_SLOW=1 (minutes each).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, REPO

PINS = os.path.join(REPO, "oracle", "pins.json")
SLOW = os.environ.get("LBM_SLOW") == "1"


def test_recorded_pins_match_known_answers():
    pins = json.load(open(PINS))
    assert set(pins) >= {"geometry", "poiseuille_converge", "ldc_serial_converge", "bif_as_shipped",
                         "bif_inlet_block1", "ldc_two_phase_converge"}
    g = pins["geometry"]
    for k, v in g["expect"].items():
        assert g[k] == v, k
    p = pins["poiseuille_converge"]
    assert p["stop_k"] == 6230 and p["nlattice"] == 214128 and p["fluid"] == 175200
    assert abs(p["uy_max"] - 0.096993) < 5e-7
    assert p["bad_reads"] == 0
    assert pins["ldc_serial_converge"]["stop_k"] == 5335
    b = pins["bif_as_shipped"]
    assert abs(b["umax"] - 3.5e-6) < 5e-8
    b = pins["bif_inlet_block1"]
    assert abs(b["umax"] - 0.224) < 5e-4
    assert abs(b["rho_min"] - 0.994) < 5e-4 and abs(b["rho_max"] - 1.141) < 5e-4


def test_geometry_pins_live(oracle):
    n, _ = oracle.index_transform(oracle.geo_poiseuille(64, 64, 64))
    assert n == 214128
    raw = oracle.read_geo_txt(os.path.join(GOLDEN, "bifurcation", "geo.txt"), 64, 83, 32)
    assert int((raw == 1).sum()) == 54388 and int((raw == 0).sum()) == 115596
    geo = oracle.geo_mask(raw)
    n, _ = oracle.index_transform(geo)
    assert n == 65820  # thesis 4.8


def _golden_cases():
    import sys
    sys.path.insert(0, os.path.join(GOLDEN))
    import make_golden
    return make_golden


@pytest.mark.parametrize("name", ["ldc16_two_phase", "ldc16_serial", "poiseuille_20x24x20", "bif_inlet_block1"])
def test_golden_vectors(oracle, name):
    mg = _golden_cases()
    meta = json.load(open(os.path.join(GOLDEN, "golden.json")))[name]
    kind, geo, tau, kw, steps = mg.case_setups()[name]
    m, (rho, ux, uy, uz, hist) = mg.run(name, kind, geo, tau, kw, steps)
    for k in ("sha256_macros_fluid", "sha256_f_fluid", "sha256_residuals", "n_fluid", "bad_reads"):
        assert m[k] == meta[k], (name, k)
    arrs = np.load(os.path.join(GOLDEN, "golden.npz"))
    if f"{name}.rho" in arrs:
        for k, a in zip(("rho", "ux", "uy", "uz"), (rho, ux, uy, uz)):
            assert np.array_equal(arrs[f"{name}.{k}"].view(np.uint32), a.view(np.uint32))


def test_ldc_orders_agree_to_race_noise(oracle):
    """The two LDC wall orders (two-phase = race-free semantics, serial = one serialisation
    of the reference's racy in-place bounce-back) differ by race noise: a few percent in the
    start-up transient measured here, 2e-4 at convergence."""
    g = oracle.geo_ldc(16, 16, 16)
    a = oracle.Oracle(oracle.LDC, g, 0.55, ldc_order=oracle.TWO_PHASE)
    b = oracle.Oracle(oracle.LDC, g, 0.55, ldc_order=oracle.SERIAL_EMU)
    a.step(40)
    b.step(40)
    fl = g == 3
    ua = np.stack(a.macros()[1:])[:, fl]
    ub = np.stack(b.macros()[1:])[:, fl]
    rel = np.linalg.norm(ua - ub) / np.linalg.norm(ua)
    assert 0 < rel < 5e-2


def test_mass_conservation_closed_box(oracle):
    """Bounce-back walls conserve mass: with the lid at rest the LDC box keeps sum(rho)."""
    g = oracle.geo_ldc(12, 12, 12)
    g[g == 2] = 1  # lid -> wall: fully closed box
    o = oracle.Oracle(oracle.LDC, g, 0.55)
    o.step(1)
    m0 = float(o.macros()[0][g == 3].astype(np.float64).sum())
    o.step(30)
    m1 = float(o.macros()[0][g == 3].astype(np.float64).sum())
    assert abs(m1 - m0) / m0 < 1e-6


@pytest.mark.skipif(not SLOW, reason="minutes: set LBM_SLOW=1")
def test_poiseuille_converge_pin(oracle):
    g = oracle.geo_poiseuille(64, 64, 64)
    o = oracle.Oracle(oracle.POISEUILLE, g, 0.58)  # the oracle's own uygt, as pin_check.py
    k, _ = o.run_converge()
    assert k == 6230
    uy = o.macros()[2]
    assert abs(float(uy[g == 4].max()) - 0.096993) < 5e-7


def test_generic_nee_matches_coronary_expressions(oracle):
    """coronary.cu writes its boundary equilibria as hand-simplified 'tmp' expressions
    (inlet 716-794 with rho 1, outlets 795-943 with rho of the fluid); the generic oracle (and
    liblbm) use feq_bc: the update kernel's feq_q in fp32 throughout.  Same bits for every u
    tried -- and the update form itself differs at q = 14 on a z face (its fp64 term)."""
    rng = np.random.default_rng(1)
    f32 = np.float32
    for u in np.concatenate([rng.uniform(-0.2, 0.2, 400), [0.1745 / 1.5441, 0.1 / 1.5441, 0.02 / 1.5441]]):
        u = f32(u)
        rho = f32(rng.uniform(0.9, 1.1))
        one = f32(1.0)
        # inlet, face +x, rho_bc = 1, u_bc = (u, 0, 0): q = 1 (w 1/18), 7, 8, 11, 12 (w 1/36)
        e = oracle.feq_bc(1.0, float(u), 0.0, 0.0)
        assert e[1] == one / f32(18) * (one + f32(3) * u + f32(3) * u * u)
        for q in (7, 8, 11, 12):
            assert e[q] == one / f32(36) * (one + f32(3) * u + f32(3) * u * u)
        # outlet, face -x, rho_bc = rho_F: q = 2, 9, 10, 13, 14
        e = oracle.feq_bc(float(rho), float(u), 0.0, 0.0)
        assert e[2] == rho / f32(18) * (one - f32(3) * u + f32(3) * u * u)
        for q in (9, 10, 13, 14):
            assert e[q] == rho / f32(36) * (one - f32(3) * u + f32(3) * u * u)
        # z outlets, face -z, u_bc = (0, 0, u): q = 6, 12, 14, 17, 18
        e = oracle.feq_bc(float(rho), 0.0, 0.0, float(u))
        assert e[6] == rho / f32(18) * (one - f32(3) * u + f32(3) * u * u)
        for q in (12, 14, 17, 18):
            assert e[q] == rho / f32(36) * (one - f32(3) * u + f32(3) * u * u)
    e_upd = oracle.feq(1.05, 0.0, 0.0, 0.0123)
    e_bc = oracle.feq_bc(1.05, 0.0, 0.0, 0.0123)
    assert np.array_equal(np.delete(e_upd, 14), np.delete(e_bc, 14))


def _cub_reduce_py(v, ipt, vec, grid_cap):
    """Independent restatement of CUB's two-pass device reduction (pure Python, fp32 via numpy
    scalars): even-share tiles of 256 * ipt items, per-thread serial folds (vectorised loads of
    full tiles, striped partial tiles), 32-lane shuffle-down warp trees, warp sums in order,
    a second single-block pass over the partials, then 0.f + S."""
    f32 = np.float32
    n = len(v)
    tile = 256 * ipt
    tiles = -(-n // tile)
    grid = 1 if tiles <= 1 else min(tiles, grid_cap)
    avg, big = tiles // grid, tiles - (tiles // grid) * grid

    def block(agg, num_valid):
        s = None
        for w in range(8):
            valid = min(32, num_valid - 32 * w)
            if valid <= 0:
                break
            lane = list(agg[32 * w:32 * w + 32])
            off = 1
            while off < 32:
                new = list(lane)
                for l in range(32):
                    if l + off < valid:
                        new[l] = f32(lane[l + off] + lane[l])
                lane = new
                off *= 2
            s = lane[0] if s is None else f32(s + lane[0])
        return s

    parts = []
    for b in range(grid):
        t0 = b * (avg + 1) if b < big else big * (avg + 1) + (b - big) * avg
        off, end = t0 * tile, min(n, (t0 + avg + (1 if b < big else 0)) * tile)
        agg = [None] * 256
        num_valid = 256
        while off + tile <= end:
            for t in range(256):
                for i in range(ipt // vec):
                    for k in range(vec):
                        x = v[off + vec * t + 256 * vec * i + k]
                        agg[t] = x if agg[t] is None else f32(agg[t] + x)
            off += tile
        if off < end:
            valid = end - off
            if agg[0] is None:
                num_valid = min(valid, 256)
            for t in range(256):
                for i in range(t, valid, 256):
                    agg[t] = v[off + i] if agg[t] is None else f32(agg[t] + v[off + i])
        parts.append(block(agg, num_valid))
    agg = [None] * 256
    for t in range(256):
        for i in range(t, grid, 256):
            agg[t] = parts[i] if agg[t] is None else f32(agg[t] + parts[i])
    return float(f32(f32(0.0) + block(agg, min(grid, 256))))


@pytest.mark.parametrize("n,ipt,vec,cap", [(5000, 16, 4, 240), (70000, 20, 2, 3), (33000, 16, 4, 5), (300, 16, 4, 240)])
def test_cub_tree_restated_twice(oracle, n, ipt, vec, cap):
    """orc_cub_reduce (the oracle's C restatement of thrust::reduce's CUB tree, the residual
    order liblbm's LBM_SUM_CUB_TREE must match) equals an independent Python restatement bit for
    bit: several tiles per block, partial last tiles, a single partial tile."""
    v = np.random.RandomState(n).rand(n).astype(np.float32) * np.float32(1e-3)
    assert np.float32(oracle.cub_reduce(v, ipt, vec, cap)) == np.float32(_cub_reduce_py(list(v), ipt, vec, cap))
