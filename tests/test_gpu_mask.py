"""geo_pre on the device (lbm_desc.mask): the codes the device builds from a raw
mask equal the oracle's restatement of bifurcation.cu:63-239 (orc_geo_mask, pinned by the
reference's geo.txt counts), cell for cell, for the shipped geometry, synthetic vessel masks of
ragged shapes, random noise masks and halo slabs; lattices built and initialised that way step
bit for bit like the oracle and like the host-ingested path."""
import numpy as np
import pytest

from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu


def vessel_mask(shape, seed, nballs=5):
    """A tube along y with random bulges, 0 on the outer x / z layers (as geo.txt)."""
    nz, ny, nx = shape
    rng = np.random.default_rng(seed)
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    r = min(nx, nz) / 3.2
    m = ((x - (nx - 1) / 2) ** 2 + (z - (nz - 1) / 2) ** 2) <= r * r
    for _ in range(nballs):
        c = rng.uniform([0, 0, 0], [nz, ny, nx])
        rr = rng.uniform(1.5, min(nx, nz) / 3)
        m |= ((z - c[0]) ** 2 + (y - c[1]) ** 2 + (x - c[2]) ** 2) <= rr * rr
    m = m.astype(np.uint8)
    m[:, :, 0] = m[:, :, -1] = 0
    m[0] = m[-1] = 0
    return m


# D3Q19 lattice vectors in the kernels' order (lbm_d3q19.hpp)
E_Q = [(0, 0, 0), (1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1), (1, 1, 0), (1, -1, 0),
       (-1, 1, 0), (-1, -1, 0), (1, 0, 1), (1, 0, -1), (-1, 0, 1), (-1, 0, -1), (0, 1, 1), (0, -1, 1),
       (0, 1, -1), (0, -1, -1)]


def defined_slots(geo, f, fluid=4):
    """The populations every storage mode and kernel path agrees on: all 19 of each fluid cell,
    and of each boundary (NEE) cell B the slots q its fluid neighbour B + e_q pulls -- the NEE
    values.  Compact rows (LBM_TUNE_COMPACT) keep no slots for the passive cells outside the row
    spans (lbm_get_f reports 0), consumer-side bounce-back never writes wall slots, and the NEE
    cells' other slots are unspecified (lanes holding an NEE cell store whole vectors for the
    directions its face does not take); lbm.h defines only the fluid cells' values."""
    fl = geo == fluid
    nee = (geo != 0) & (geo != -1) & (geo != 1) & ~fl
    out = [f[:, fl].ravel()]
    for q, (ex, ey, ez) in enumerate(E_Q):
        if q == 0:
            continue
        pulled = np.roll(fl, (-ez, -ey, -ex), axis=(0, 1, 2))  # B + e_q is fluid
        out.append(f[q][nee & pulled])
    return np.concatenate(out)


def inlet_tables(shape, seed):
    nz, ny, nx = shape
    rng = np.random.default_rng(seed)
    return (rng.uniform(0.01, 0.05, (nz, nx)).astype(np.float32),
            rng.uniform(0.01, 0.05, (nz, nx)).astype(np.float32))


def test_device_geo_bifurcation(gpu, oracle):
    from lbm_amd import cases
    lat, raw = cases.bifurcation_device(1)
    want = oracle.geo_mask(raw)
    got = lat.geo()
    assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} codes differ"
    # the host-ingested context reports the codes it was given
    host, geo, _, _ = cases.bifurcation(1)
    assert np.array_equal(host.geo(), geo)
    assert lat.counts() == host.counts()


@pytest.mark.parametrize("shape", [(23, 31, 37), (12, 9, 13), (30, 40, 66)])
def test_device_geo_vessels_and_noise(gpu, oracle, shape, row_axis):
    from lbm_amd import cases
    for raw in (vessel_mask(shape, 1), (np.random.default_rng(2).random(shape) < 0.75).astype(np.uint8)):
        lat = cases.mask_device(raw)
        want = oracle.geo_mask(raw.astype(np.int32))
        got = lat.geo()
        assert np.array_equal(got, want), f"{shape}: {np.count_nonzero(got != want)} codes differ"
        lat.close()


@pytest.mark.parametrize("shape", [(23, 31, 37), (30, 40, 66)])
def test_device_mask_lattice_bitwise(gpu, oracle, shape, cells_per_lane, row_axis):
    """Device codes + device initialize() vs the oracle (and the host path) over 60 steps."""
    from lbm_amd import cases, geo_mask, initial_fields, Lattice, LBM_CASE_MASK, LBM_INIT_EXPANDED
    raw = vessel_mask(shape, 3)
    inl, outl = inlet_tables(shape, 4)
    dev = cases.mask_device(raw, inl, outl, tau=0.55)
    geo = geo_mask(raw.astype(np.int32))
    assert np.array_equal(dev.geo(), geo)
    inl_m = np.where(geo[:, 1, :] == 2, inl, 0).astype(np.float32)
    outl_m = np.where(geo[:, -2, :] == 3, outl, 0).astype(np.float32)
    host = Lattice(LBM_CASE_MASK, shape, 0.55, geo, inlet_uy=inl_m)
    host.init_equilibrium(LBM_INIT_EXPANDED, *initial_fields(2, geo, inl_m, outl_m))
    o = oracle.Oracle(oracle.MASK, geo, 0.55, inlet_uy=inl_m, outlet_uy=outl_m)
    for s in (1, 59):
        hd, hh = dev.step(s), host.step(s)
        o.step(s)
        assert np.array_equal(hd.view(np.uint32), hh.view(np.uint32))
        assert_bitwise(dev, o, geo, 2, f"device mask {shape}")
    fd, fh = dev.f(), host.f()
    m = geo == 4
    assert np.array_equal(fd[:, m].view(np.uint32), fh[:, m].view(np.uint32))


def test_device_bifurcation_matches_host(gpu):
    from lbm_amd import cases
    dev, _ = cases.bifurcation_device(1)
    host, geo, _, _ = cases.bifurcation(1)
    hd, hh = dev.step(300), host.step(300)
    assert np.array_equal(hd.view(np.uint32), hh.view(np.uint32))
    for a, b in zip(dev.macros(), host.macros()):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("nslabs", [2, 3])
def test_device_mask_slabs(gpu, nslabs, row_axis):
    """Halo slabs built from slab_mask (3 extra planes each side): each slab's codes are the
    global codes of its planes, and the loopback slab run equals the single domain."""
    from lbm_amd import cases, geo_mask, x_align_for, LBM_CASE_MASK
    import lbm_amd
    shape = (29, 31, 37)
    nz = shape[0]
    raw = vessel_mask(shape, 5)
    inl, outl = inlet_tables(shape, 6)
    geo = geo_mask(raw.astype(np.int32))
    one = cases.mask_device(raw, inl, outl)
    xa = x_align_for(geo, LBM_CASE_MASK)
    slabs = []
    for i in range(nslabs):
        z0, z1 = cases.slab_bounds(nz, nslabs, i)
        lat = cases.mask_device(cases.slab_mask(raw, z0, z1), inl, outl, z_offset=z0, nz_global=nz,
                                halo_planes=True, x_align=xa)
        assert np.array_equal(lat.geo(), geo[z0:z1]), f"slab {i} codes"
        slabs.append((z0, z1, lat))
    h1 = one.step(40)
    hs = lbm_amd.group_step([s[2] for s in slabs], 40)
    np.testing.assert_allclose(hs, h1, rtol=0, atol=1e-6)
    ref = one.macros()
    for z0, z1, lat in slabs:
        for a, b in zip(lat.macros(), ref):
            assert np.array_equal(a.view(np.uint32), b[z0:z1].view(np.uint32))


def test_bifurcation_upsampled_bitwise(gpu, oracle):
    """SURVEY 8(d) C4's bandwidth-relevant sparse variant (the shipped mask upsampled 4x per
    axis, 256 x 332 x 128, ~4 M stored cells; the bench's secondary line): device codes equal the
    oracle's geo_pre, and the lattice steps bit for bit like the oracle."""
    from lbm_amd import cases, index_transform
    lat, up = cases.bifurcation_upsampled(4)
    shape = lat.launch_shape()  # half-empty chunks: compact lists of 4-cell groups (LBM_TUNE_GROUPS auto)
    assert shape["cells_per_lane"] == 4 and shape["grid_stride"] == 2, shape
    geo = oracle.geo_mask(up.astype(np.int32))
    got = lat.geo()
    assert np.array_equal(got, geo), f"{np.count_nonzero(got != geo)} codes differ"
    nl, _ = index_transform(geo)
    assert 3_500_000 < nl < 4_500_000, nl  # "~4 M stored cells" 
    from lbm_amd import read_bc_txt, BIF_SHAPE
    import os
    _, inl, outl = read_bc_txt(os.path.join(cases.BIF_DIR, "bc.txt"), tuple(BIF_SHAPE), 1)
    inl4 = inl.repeat(4, 0).repeat(4, 1)
    outl4 = outl.repeat(4, 0).repeat(4, 1)
    inl_m = np.where(geo[:, 1, :] == 2, inl4, 0).astype(np.float32)
    outl_m = np.where(geo[:, -2, :] == 3, outl4, 0).astype(np.float32)
    o = oracle.Oracle(oracle.MASK, geo, 0.55, inlet_uy=inl_m, outlet_uy=outl_m)
    for s in (1, 9):
        lat.step(s)
        o.step(s)
        assert_bitwise(lat, o, geo, 2, f"bif x4 +{s}")
    assert o.bad_reads() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["pipe", "bif_x4"])
def test_grid_stride_bitwise(gpu, knob, case):
    """LBM_TUNE_GRID_STRIDE changes only which wave takes which chunk.  A pipe (a sparse chunk
    list whose lanes are nearly all busy: one chunk per wave by default) with the loop forced on,
    and the upsampled bifurcation (half-empty chunks: the loop by default) forced off and on,
    step bit for bit like their defaults.  The defaults are pinned to the oracle by the tests
    above and by test_gpu_parity.py."""
    from lbm_amd import cases
    knob(gpu.TUNE_CELLS_PER_LANE, 4)
    knob(gpu.TUNE_GROUPS, 1)  # chunk waves (the group lists have their own test below)
    knob(gpu.TUNE_ROW_AXIS, 2)  # rows along the pipe: one chunk per (x, z) column, lanes full

    def run(v):
        with gpu.tuned(gpu.TUNE_GRID_STRIDE, v):
            lat = cases.poiseuille(64, 256, 64)[0] if case == "pipe" else cases.bifurcation_upsampled(4)[0]
        shape = lat.launch_shape()
        hist = lat.step(12)
        f = lat.f()
        lat.close()
        return shape, f, hist

    s0, f0, h0 = run(0)
    assert s0["grid_stride"] == (1 if case == "bif_x4" else 0), s0
    for v in ((1, 2) if case == "pipe" else (1, 2, 3)):
        s, f, h = run(v)
        assert s["grid_stride"] == (0 if v == 1 else 1), (v, s)
        assert np.array_equal(f.view(np.uint32), f0.view(np.uint32)), f"{case} grid_stride={v}"
        # the residual's fp64 |u| sum is accumulated per block, so the launch shape may move its
        # last bits: the fp32 sums S_k agree to an ulp, the residuals to ~1e-7 absolute (lbm.h)
        assert np.all(np.isfinite(h)) and np.allclose(h, h0, rtol=0, atol=2e-7), (v, h, h0)


@pytest.mark.gpu
@pytest.mark.parametrize("lattice", ["pipe_y", "pipe_y_stride", "ldc", "coronary"])
def test_xcd_run_bitwise(gpu, knob, lattice):
    """LBM_TUNE_XCD_RUN changes only which XCD takes which chunk workgroup: a pipe with rows along
    y (runs of eight by default), a cavity (one eighth per XCD by default) and the coronary tree
    (compact one-cell waves, runs of four by default) under both orders and runs of 16 workgroups
    step bit for bit alike, residual histories included (each partial slot sums the same chunks
    whatever the order).  The pipe's grid-stride loop (LBM_TUNE_GRID_STRIDE 2), whose waves take
    their chunks by XCD and round whatever the order, ignores the knob: same partial slots, same
    residual bits."""
    from lbm_amd import cases
    if lattice != "coronary":
        knob(gpu.TUNE_CELLS_PER_LANE, 4)
    if lattice == "pipe_y_stride":
        knob(gpu.TUNE_GRID_STRIDE, 2)

    def run(v):
        with gpu.tuned(gpu.TUNE_XCD_RUN, v):
            if lattice.startswith("pipe_y"):
                lat = cases.poiseuille(40, 512, 36)[0]
                assert lat.launch_shape()["grid_stride"] == (1 if lattice == "pipe_y_stride" else 0)
            elif lattice == "ldc":
                lat = cases.ldc_device(96, 96, 96)
            else:
                lat = cases.coronary(cases.coronary_reference_vessel())[0]
        hist = lat.step(9)
        f = lat.f()
        lat.close()
        return f, hist

    f0, h0 = run(0)
    for v in (17, 1, 5):
        f, h = run(v)
        assert np.array_equal(f.view(np.uint32), f0.view(np.uint32)), f"{lattice} xcd_run={v}"
        assert np.array_equal(h.view(np.uint32), h0.view(np.uint32)), (v, h, h0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["bif_x4", "coronary", "pipe"])
def test_groups_bitwise(gpu, knob, case):
    """LBM_TUNE_GROUPS changes only which lane updates which cells: the upsampled bifurcation and
    the coronary tree (compact 4-cell group lists by default) with the lists off, and a pipe
    (whole chunks by default) with them forced on, step bit for bit like their defaults --
    which the oracle pins (test_bifurcation_upsampled_bitwise, tests with the cells_per_lane
    fixture's "4groups" path)."""
    from lbm_amd import cases
    knob(gpu.TUNE_CELLS_PER_LANE, 4)

    def build():
        if case == "bif_x4":
            return cases.bifurcation_upsampled(4)[0]
        if case == "coronary":
            return cases.coronary(cases.coronary_reference_vessel())[0]
        return cases.poiseuille(64, 256, 64)[0]

    def run(v):
        with gpu.tuned(gpu.TUNE_GROUPS, v):
            lat = build()
        shape = lat.launch_shape()
        hist = lat.step(12)
        f = defined_slots(lat.geo(), lat.f())
        lat.close()
        return shape, f, hist

    s0, f0, h0 = run(0)
    assert s0["grid_stride"] == (0 if case == "pipe" else 2), s0
    s1, f1, h1 = run(2 if case == "pipe" else 1)
    assert s1["grid_stride"] == (2 if case == "pipe" else 1), s1
    assert np.array_equal(f1.view(np.uint32), f0.view(np.uint32)), case
    # per-block fp64 partials: the launch shape may move the residual's last bits (lbm.h)
    assert np.all(np.isfinite(h1)) and np.allclose(h1, h0, rtol=0, atol=2e-7), (h1, h0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["coronary", "bif"])
def test_one_cell_groups_default_bitwise(gpu, knob, case):
    """A sparse list with few active groups (the coronary tree; C4, whose 391 chunks are one-cell
    size anyway) runs one cell per lane by default, over consecutive cells of its compact rows.
    Forcing four cells per lane over the compact group list, or one cell per lane over whole
    chunks of the dense box, changes only which lane updates which cell: populations bit for
    bit equal."""
    from lbm_amd import cases

    def build():
        if case == "coronary":
            return cases.coronary(cases.coronary_reference_vessel())[0]
        return cases.bifurcation(1)[0]

    def run(cpl, groups):
        with gpu.tuned(gpu.TUNE_CELLS_PER_LANE, cpl), gpu.tuned(gpu.TUNE_GROUPS, groups):
            lat = build()
        shape = lat.launch_shape()
        hist = lat.step(12)
        f = defined_slots(lat.geo(), lat.f())
        lat.close()
        return shape, f, hist

    s0, f0, h0 = run(0, 0)  # compact rows, one cell per lane, no list (LBM_TUNE_COMPACT auto)
    assert s0["cells_per_lane"] == 1 and s0["grid_stride"] == 3, s0
    for cpl, groups, want in ((4, 2, (4, 2)), (1, 1, (1, 0))):
        s, f, h = run(cpl, groups)
        assert (s["cells_per_lane"], s["grid_stride"]) == want, (cpl, groups, s)
        assert np.array_equal(f.view(np.uint32), f0.view(np.uint32)), (case, cpl, groups)
        assert np.all(np.isfinite(h)) and np.allclose(h, h0, rtol=0, atol=2e-7), (h, h0)


@pytest.mark.parametrize("case", ["bif", "bif_x2_device", "coronary", "vessel_x"])
def test_compact_rows_vs_dense(gpu, knob, case, tmp_path):
    """Compact rows (LBM_TUNE_COMPACT, the default for sparse single-domain lattices: every
    storage row keeps only the span of its stored cells) against the dense box: the same fields
    and populations bit for bit after stepping, residuals to one fp32 ulp of S (the |u| partials
    are summed per launch block, and the blocks differ), a checkpoint resumed bit for bit, and
    the buffers a fraction of the box."""
    from lbm_amd import cases
    import lbm_amd

    def make(compact):
        # the bifurcations take compact rows by default (auto); the small trees are forced
        # onto group lists (LBM_TUNE_GROUPS 2) and compact rows (LBM_TUNE_COMPACT 2)
        forced = case in ("coronary", "vessel_x")
        knob(lbm_amd.TUNE_GROUPS, 2 if forced else 0)
        knob(lbm_amd.TUNE_COMPACT, (2 if forced else 0) if compact else 1)
        if case == "bif":
            return cases.bifurcation(1)[0]
        if case == "bif_x2_device":
            return cases.bifurcation_upsampled(2)[0]
        if case == "coronary":
            return cases.coronary(*cases.coronary_small_vessel())[0]
        return cases.mask_device(np.ascontiguousarray(vessel_mask((30, 40, 66), 3).transpose(0, 2, 1)))

    a, b = make(True), make(False)
    sa, sb = a.storage(), b.storage()
    assert sa["compact"] and not sb["compact"], (sa, sb)
    assert sa["cells"] < 0.6 * sb["cells"], (sa, sb)
    ha, hb = a.step(25), b.step(25)
    np.testing.assert_allclose(np.asarray(ha, np.float64), np.asarray(hb, np.float64), rtol=0, atol=1.2e-7)
    geo = b.geo()
    fl = geo == 4
    for x, y in zip(a.macros(), b.macros()):
        assert np.array_equal(x[fl].view(np.uint32), y[fl].view(np.uint32))
    fa, fb = a.f(), b.f()
    assert np.array_equal(fa[:, fl].view(np.uint32), fb[:, fl].view(np.uint32))
    path = str(tmp_path / "compact.ckpt")
    a.checkpoint_save(path)
    ha2 = a.step(10)
    c = make(True)
    c.checkpoint_load(path)
    hc = c.step(10)
    assert np.array_equal(ha2.view(np.uint32), hc.view(np.uint32))
    for x, y in zip(a.macros(), c.macros()):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    with pytest.raises(lbm_amd.LbmError):  # a compact lattice is a single domain
        a.attach_rccl(lbm_amd.rccl_unique_id(), 0, 1)
    for lat in (a, b, c):
        lat.close()


@pytest.mark.parametrize("path", ["bif_1cell_compact", "bif_4cell_compact", "ldc_1cell_box"])
def test_consumer_side_steps_write_no_wall_slot(gpu, knob, path):
    """With bounce-back on the consumer side no wall slot is read, and no step stores into one
    except where a 4-cell lane stores its whole 16-B vector over a 4-cell group that also holds a
    fluid cell (the wall cells' slots in that group take the lane's values; nothing reads them).
    Every other wall slot keeps the sentinel it was set to -- one-cell lanes store cell by cell, so
    there that is every wall slot -- and so no store of a lane strays into another group or row
    (the check defined_slots cannot make, since it compares only the slots the modes agree on;
    ADVICE r04)."""
    from lbm_amd import cases
    import lbm_amd
    four = path == "bif_4cell_compact"
    if four:
        knob(lbm_amd.TUNE_CELLS_PER_LANE, 4)
        knob(lbm_amd.TUNE_GROUPS, 2)
        knob(lbm_amd.TUNE_COMPACT, 2)
    if path.startswith("bif"):
        lat, geo, _, _ = cases.bifurcation(1)
        assert lat.storage()["compact"]
        fluid, steps = geo == 4, 24
    else:
        lat = cases.ldc_device(32, 32, 32)
        geo = lat.geo()
        fluid, steps = geo == 3, 23  # odd: buffer 1, which the initial bounce-back priming of buffer 0 never touched
    assert lat.launch_shape()["cells_per_lane"] == (4 if four else 1)
    wall = geo == 1
    if four:  # wall cells whose storage group (4 cells along the row, xshift applied) holds no fluid cell
        lay = lat.layout()
        ax = 2 if lay["row_axis"] == 1 else 1  # raster axis of the rows: x (2) or y (1)
        pos = np.arange(geo.shape[ax]) - (lay["x_align"] - 1)
        grp = np.floor_divide(pos, 4)
        shape = [1, 1, 1]
        shape[ax] = -1
        g = np.broadcast_to(grp.reshape(shape), geo.shape)
        fl = np.moveaxis(fluid, ax, -1)
        gg = np.moveaxis(g, ax, -1)
        has = np.zeros_like(fl)
        for k in np.unique(grp):
            sel = gg == k
            any_fl = (fl & sel).any(axis=-1, keepdims=True)
            has |= sel & any_fl
        wall &= ~np.moveaxis(has, -1, ax)
        assert wall.sum() > 1000
    f = lat.f()
    # distinct small values (the first step of the bifurcation pulls its walls raw)
    sentinel = (0.01 + (np.arange(wall.sum() * 19).reshape(19, -1) % 1021) * 1e-5).astype(np.float32)
    f[:, wall] = sentinel
    lat.set_f(f)
    lat.step(steps, history=False)
    got = lat.f()[:, wall]
    assert np.all(np.isfinite(lat.macros()[0][fluid]))
    bad = np.count_nonzero(got.view(np.uint32) != sentinel.view(np.uint32))
    assert bad == 0, f"{path}: {bad} wall slots written"
    lat.close()


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["bif_1cell_compact", "bif_4cell_compact", "coronary_1cell_compact", "ldc_1cell_box",
                                  "pipe_producer"])
def test_consumer_side_steps_read_no_wall_slot(gpu, knob, path):
    """The property the no-write check above stands in for, tested directly: with bounce-back on
    the consumer side no step after the first reads a wall slot.  Two identical lattices step
    once; then every slot of every wall cell of both buffers of one of them becomes a quiet NaN
    (lbm_debug_poison_walls: the wall slots whole 16-B stores cover included) and both step on --
    fields, populations of the fluid cells and residuals stay bit for bit equal.  A lattice that
    bounces back on the producer side pulls the NaNs at once, which shows the poison reaches
    every wall slot a step could read."""
    from lbm_amd import cases
    import lbm_amd
    if path == "bif_4cell_compact":
        knob(lbm_amd.TUNE_CELLS_PER_LANE, 4)
        knob(lbm_amd.TUNE_GROUPS, 2)
        knob(lbm_amd.TUNE_COMPACT, 2)

    def make():
        if path.startswith("bif"):
            return cases.bifurcation(1)[0]
        if path.startswith("coronary"):
            raw, ends = cases.coronary_small_vessel()
            return cases.coronary(raw, ends)[0]
        if path == "ldc_1cell_box":
            return cases.ldc_device(32, 32, 32)
        return cases.poiseuille(20, 28, 20)[0]

    a, b = make(), make()
    if path != "pipe_producer":
        assert a.launch_shape()["cells_per_lane"] == (4 if path == "bif_4cell_compact" else 1)
    geo = a.geo()
    fluid = geo == (3 if path.startswith("ldc") else 4)
    a.step(1)
    b.step(1)
    b.debug_poison_walls()
    ha, hb = a.step(25), b.step(25)
    mb = np.stack(b.macros())[:, fluid]
    if path == "pipe_producer":
        assert not np.all(np.isfinite(mb)), "the poisoned wall slots never reached a fluid cell"
        return
    ma = np.stack(a.macros())[:, fluid]
    assert np.array_equal(ma.view(np.uint32), mb.view(np.uint32)), f"{path}: fields differ after poisoning the walls"
    assert np.array_equal(a.f()[:, fluid].view(np.uint32), b.f()[:, fluid].view(np.uint32))
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32))
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["bif_x4", "pipe"])
def test_nee_order_bitwise(gpu, knob, case):
    """LBM_TUNE_NEE_ORDER moves only where the NEE blocks are dispatched (trailing the grid-stride
    group lists by default, leading the pipe's chunk list): both orders step bit for bit alike,
    residual histories included -- the blocks keep their logical places and partial slots."""
    from lbm_amd import cases
    knob(gpu.TUNE_CELLS_PER_LANE, 4)

    def run(order):
        with gpu.tuned(gpu.TUNE_NEE_ORDER, order):
            lat = cases.bifurcation_upsampled(4)[0] if case == "bif_x4" else cases.poiseuille(40, 300, 36)[0]
        assert lat.nee_path()["path"] == "blocks"
        h = lat.step(11)
        f = lat.f()
        lat.close()
        return f, h

    f0, h0 = run(0)
    for order in (1, 2):
        f, h = run(order)
        assert np.array_equal(f.view(np.uint32), f0.view(np.uint32)), f"{case} nee order {order}"
        assert np.array_equal(h.view(np.uint32), h0.view(np.uint32)), (order, h, h0)
