"""Checkpoint / resume (lbm_checkpoint_save / lbm_checkpoint_load; SURVEY.md section 5: the
reference cannot restart a run).  A run saved after k steps and resumed in a fresh context
continues bit for bit: populations, macros (the lazy read-out right after the load included),
the residual history and the convergence state -- on every boundary kind whose state is more
than the populations (the NEE-adjacent cells' previous (rho, u)), on both step paths, and for
z-slabs stepped together."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(a, b, what):
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), what


def _builders():
    from lbm_amd import cases
    raw, ends = cases.coronary_small_vessel()
    return {
        "ldc": lambda: cases.ldc(24)[0],
        "poiseuille": lambda: cases.poiseuille(20, 28, 20)[0],
        "bifurcation": lambda: cases.bifurcation(1)[0],
        "coronary": lambda: cases.coronary(raw, ends)[0],
    }


@pytest.mark.parametrize("case", ["ldc", "poiseuille", "bifurcation", "coronary"])
def test_resume_is_bitwise(gpu, tmp_path, cells_per_lane, case):
    make = _builders()[case]
    a = make()
    a.step(7)
    path = str(tmp_path / "ck.bin")
    a.checkpoint_save(path)
    ha = a.step(25)
    b = make()
    b.checkpoint_load(path)
    hb = b.step(25)
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32)), f"{case}: residual histories differ"
    _same(a.macros(), b.macros(), f"{case}: macros differ after resuming")
    assert np.array_equal(a.f().view(np.uint32), b.f().view(np.uint32)), f"{case}: populations differ"
    assert a.state()["k"] == b.state()["k"] == 32
    a.close()
    b.close()


def test_resume_macros_right_after_load(gpu, tmp_path):
    from lbm_amd import cases
    a, geo, _, _ = cases.bifurcation(1)
    a.step(11)
    path = str(tmp_path / "ck.bin")
    a.checkpoint_save(path)
    b, _, _, _ = cases.bifurcation(1)
    b.checkpoint_load(path)
    _same(a.macros(), b.macros(), "lazy macro read-out after a load")
    a.close()
    b.close()


def test_resume_under_convergence_control(gpu, tmp_path):
    """Saved mid-run with the stopping rule on: the resumed run stops at the same step."""
    from lbm_amd import cases
    a = cases.ldc(16)[0]
    a.set_convergence(True, 10000, 50, 1e-6)
    a.step(300, history=False)
    path = str(tmp_path / "ck.bin")
    a.checkpoint_save(path)
    a.step(10001, history=False)
    sa = a.state()
    b = cases.ldc(16)[0]
    b.set_convergence(True, 10000, 50, 1e-6)
    b.checkpoint_load(path)
    b.step(10001, history=False)
    sb = b.state()
    assert sa["stopped"] == sb["stopped"] == 1 and sa["k"] == sb["k"] and sa["residual"] == sb["residual"]
    _same(a.macros(), b.macros(), "converged fields")
    a.close()
    b.close()


def test_resume_slabs(gpu, tmp_path):
    """Three z-slabs stepped together (lbm_group_step), one file per slab."""
    from lbm_amd import cases, initial_fields, Lattice, LBM_CASE_POISEUILLE, LBM_INIT_EXPANDED
    import lbm_amd
    nx, ny, nz = 24, 30, 33
    _, geo = cases.poiseuille(nx, ny, nz)
    prof = lbm_amd.poiseuille_profile(nx, nz)
    rho, ux, uy, uz = initial_fields(1, geo)
    xa = lbm_amd.x_align_for(geo, LBM_CASE_POISEUILLE)

    def slabs():
        out = []
        for i in range(3):
            z0, z1 = cases.slab_bounds(nz, 3, i)
            lat = Lattice(LBM_CASE_POISEUILLE, (z1 - z0, ny, nx), 0.58, cases.slab_geo(geo, z0, z1),
                          halo_planes=True, inlet_uy=prof, outlet_uy=prof, z_offset=z0, nz_global=nz, x_align=xa)
            lat.init_equilibrium(LBM_INIT_EXPANDED, rho[z0:z1], ux[z0:z1], uy[z0:z1], uz[z0:z1])
            out.append(lat)
        return out

    a = slabs()
    lbm_amd.group_step(a, 9)
    for i, lat in enumerate(a):
        lat.checkpoint_save(str(tmp_path / f"ck{i}.bin"))
    ha = lbm_amd.group_step(a, 30)
    b = slabs()
    for i, lat in enumerate(b):
        lat.checkpoint_load(str(tmp_path / f"ck{i}.bin"))
    hb = lbm_amd.group_step(b, 30)
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32))
    for x, y in zip(a, b):
        _same(x.macros(), y.macros(), "slab macros")
        x.close()
        y.close()


def test_load_rejects_other_lattices(gpu, tmp_path):
    from lbm_amd import cases
    import lbm_amd
    a = cases.ldc(24)[0]
    a.step(3)
    path = str(tmp_path / "ck.bin")
    a.checkpoint_save(path)
    for other in (cases.ldc(20)[0], cases.ldc(24, tau=0.6)[0], cases.poiseuille(24, 24, 24)[0]):
        with pytest.raises(lbm_amd.LbmError):
            other.checkpoint_load(path)
        other.close()
    (tmp_path / "short.bin").write_bytes(open(path, "rb").read()[:4096])
    with pytest.raises(lbm_amd.LbmError):
        a.checkpoint_load(str(tmp_path / "short.bin"))
    with pytest.raises(lbm_amd.LbmError):
        a.checkpoint_load(str(tmp_path / "missing.bin"))
    a.close()


def test_resume_rccl_slab(gpu, tmp_path):
    """A slab context on a one-rank RCCL communicator (the multi-GPU step sequence: edge and
    interior launches, parity-slot reduction, all-reduce, finisher) saved and resumed."""
    from lbm_amd import cases
    import lbm_amd

    def make():
        lat = cases.ldc_device(32, 32, 32, z_offset=32, nz_global=96)
        lat.attach_rccl(lbm_amd.rccl_unique_id(), 0, 1)
        return lat

    a = make()
    a.step(6)
    path = str(tmp_path / "ck.bin")
    a.checkpoint_save(path)
    ha = a.step(20)
    b = make()
    b.checkpoint_load(path)
    hb = b.step(20)
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32))
    _same(a.macros(), b.macros(), "RCCL slab macros")
    a.close()
    b.close()


@pytest.mark.parametrize("saved_on", [True, False])
def test_load_keeps_this_contexts_convergence_settings(gpu, tmp_path, saved_on):
    """The file supplies the run state (k, tol_count, residual, sums, stop flag); the
    convergence settings stay the loading context's own, and its step kernels follow them: a
    checkpoint saved with convergence control on loads into a context without it and keeps
    stepping (and the reverse stops at the loading context's max_it)."""
    from lbm_amd import cases
    a = cases.ldc(20)[0]
    if saved_on:
        a.set_convergence(True, max_it=12, stag_max=50, tol=1e-6)
    a.step(10)
    path = str(tmp_path / "ck.bin")
    a.checkpoint_save(path)
    b = cases.ldc(20)[0]
    if not saved_on:
        b.set_convergence(True, max_it=12, stag_max=50, tol=1e-6)
    b.checkpoint_load(path)
    b.step(20)
    st = b.state()
    if saved_on:   # b has no convergence control: all 20 steps run
        assert st["k"] == 30 and st["stopped"] == 0, st
    else:          # b stops once k > max_it = 12
        assert st["k"] == 13 and st["stopped"] == 1, st
    a.close()
    b.close()


def test_load_rejects_corrupt_header(gpu, tmp_path):
    """A header whose run state is out of range (buffer index, step count, flags) is refused
    with LBM_ERR_ARG before anything is copied to the device."""
    import struct
    from lbm_amd import cases, LbmError
    a = cases.ldc(16)[0]
    a.step(3)
    path = tmp_path / "ck.bin"
    a.checkpoint_save(str(path))
    raw = bytearray(path.read_bytes())
    # CkptHeader: magic[8], then int32 version, nx, ny, nz, z_offset, nz_global, case_kind, swap,
    # pitch, xshift, steps_done, cur, ...
    cur_at = 8 + 4 * 11
    assert struct.unpack_from("<i", raw, cur_at)[0] in (0, 1)
    for at, val in ((cur_at, 7), (cur_at - 4, -2), (cur_at - 4, 4)):  # cur, steps_done < 0, k != steps_done
        bad = bytearray(raw)
        struct.pack_into("<i", bad, at, val)
        p = tmp_path / f"bad{at}_{val}.bin"
        p.write_bytes(bytes(bad))
        b = cases.ldc(16)[0]
        with pytest.raises(LbmError, match="corrupt header"):
            b.checkpoint_load(str(p))
        b.close()
    a.close()


def _as_version2(v3: bytes) -> bytes:
    """A version-3 file of a producer-side context rewritten in round 4's version-2 layout:
    the header without walls_stale (CkptHeader: magic[8], 12 int32 from version to cur,
    halo_primed, walls_stale, tau_bits, 4 B padding, int64 ncell, buf_floats, ConvState (72 B);
    version 2: halo_primed, tau_bits, then the int64s at once)."""
    import struct
    assert struct.unpack_from("<i", v3, 60)[0] == 0  # walls_stale: producer side
    body = v3[160:]
    return v3[:8] + struct.pack("<i", 2) + v3[12:60] + v3[64:68] + v3[72:160] + body


def test_load_version2_file(gpu, tmp_path):
    """Round 4's checkpoint format (version 2, no walls_stale field) still loads: as a file whose
    wall slots were written by the steps, and the resumed run continues bit for bit.  Any other
    version is refused by number."""
    import struct
    from lbm_amd import cases, LbmError
    a = cases.poiseuille(20, 28, 20)[0]
    a.step(7)
    p3 = tmp_path / "v3.bin"
    a.checkpoint_save(str(p3))
    ha = a.step(12)
    raw = p3.read_bytes()
    p2 = tmp_path / "v2.bin"
    p2.write_bytes(_as_version2(raw))
    b = cases.poiseuille(20, 28, 20)[0]
    b.checkpoint_load(str(p2))
    hb = b.step(12)
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32))
    assert np.array_equal(a.f().view(np.uint32), b.f().view(np.uint32))
    bad = bytearray(raw)
    struct.pack_into("<i", bad, 8, 9)
    p9 = tmp_path / "v9.bin"
    p9.write_bytes(bytes(bad))
    with pytest.raises(LbmError, match="unsupported checkpoint version 9"):
        b.checkpoint_load(str(p9))
    a.close()
    b.close()


@pytest.mark.parametrize("save_box,load_box", [(0, 1), (1, 0)], ids=["consumer_to_producer", "producer_to_consumer"])
@pytest.mark.parametrize("steps", [1, 7])
def test_resume_across_bounce_back_modes(gpu, tmp_path, knob, save_box, load_box, steps):
    """The one-cell device cavity bounces back on the consumer side (no step writes a wall slot);
    its LBM_TUNE_BOX = 1 twin bounces back on the producer side and pulls the wall slots.  A file
    saved by either resumes in the other bit for bit: the header records the saver's mode, and a
    producer-side loader restores the wall slots of both buffers (the next step's source and the
    last step's, which the lazy macros read) before anything pulls them."""
    from lbm_amd import cases
    import lbm_amd

    def make(box):
        with lbm_amd.tuned(lbm_amd.TUNE_BOX, box):
            return cases.ldc_device(32, 32, 32)

    a = make(save_box)
    assert a.launch_shape()["cells_per_lane"] == 1
    a.step(steps)
    path = str(tmp_path / "ck.bin")
    a.checkpoint_save(path)
    b = make(load_box)
    b.checkpoint_load(path)
    _same(a.macros(), b.macros(), "macros right after the load")
    ha, hb = a.step(20), b.step(20)
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32)), "residual histories differ"
    _same(a.macros(), b.macros(), "macros after 20 more steps")
    a.close()
    b.close()


@pytest.mark.parametrize("steps", [1, 9])
def test_attach_after_consumer_side_steps(gpu, steps):
    """A single-domain one-cell cavity steps consumer-side, then attaches a one-rank RCCL
    communicator (producer-side slab sequence from then on): the macros read right after the
    attach, and every later step, equal those of a context that was never attached."""
    from lbm_amd import cases
    import lbm_amd
    a = cases.ldc_device(32, 32, 32)
    b = cases.ldc_device(32, 32, 32)
    a.step(steps)
    b.step(steps)
    b.attach_rccl(lbm_amd.rccl_unique_id(), 0, 1)
    _same(a.macros(), b.macros(), "macros right after the attach")
    ha, hb = a.step(15), b.step(15)
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32)), "residual histories differ"
    _same(a.macros(), b.macros(), "macros after stepping the slab sequence")
    a.close()
    b.close()


def test_group_step_after_consumer_side_steps(gpu):
    """lbm_group_step runs a context's slab ranges producer-side: a whole-domain context that
    stepped consumer-side first gets its wall slots back, and the loopback step of that one
    'slab' equals the single-domain step."""
    from lbm_amd import cases
    import lbm_amd
    a = cases.ldc_device(32, 32, 32)
    b = cases.ldc_device(32, 32, 32)
    a.step(5)
    b.step(5)
    ha = a.step(12)
    hb = lbm_amd.group_step([b], 12)
    assert np.allclose(ha, hb, rtol=0, atol=2e-7)  # per-block partials: the launch shape may move last bits
    _same(a.macros(), b.macros(), "macros after the loopback steps")
    a.close()
    b.close()


@pytest.mark.parametrize("modes", [(2, 2), (2, 1), (1, 2), (2, 3)], ids=["rec_rec", "rec_blocks", "blocks_rec", "rec_fix"])
def test_resume_nee_records(gpu, tmp_path, knob, modes):
    """A pipe whose NEE values travel as NEE records (LBM_TUNE_NEE_FIX 2: the NEE cells' slots are
    never written while stepping): the file holds the values in those slots (save puts them
    there), so it resumes bit for bit in a context of any NEE mode, and a records context takes
    its next step's values back from the loaded slots."""
    from lbm_amd import cases
    import lbm_amd
    knob(lbm_amd.TUNE_CELLS_PER_LANE, 4)

    def make(mode):
        with lbm_amd.tuned(lbm_amd.TUNE_NEE_FIX, mode):
            return cases.poiseuille(20, 512, 18)[0]

    a = make(modes[0])
    a.step(9)
    path = str(tmp_path / "ck.bin")
    a.checkpoint_save(path)
    b = make(modes[1])
    b.checkpoint_load(path)
    _same(a.macros(), b.macros(), "macros right after the load")
    ha, hb = a.step(21), b.step(21)
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32)), "residual histories differ"
    _same(a.macros(), b.macros(), "macros after 21 more steps")
    a.close()
    b.close()
