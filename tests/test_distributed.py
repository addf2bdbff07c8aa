"""N > 1 host logic on CPU: two gloo ranks run bench.py's coordination path (lbm_amd.dist) --
slab planning, the 128-byte communicator-id hand-out, max/sum reductions -- and check that
the slab masks with their halo planes tile the global lattice exactly as the halo exchange
assumes (ghost plane below = the neighbour's top plane and vice versa)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "lattice-boltzmann-method-gpu_amd"))
    import lbm_amd
    from lbm_amd import cases
    from lbm_amd import dist as ldist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    nx, ny, nz = 20, 24, 23
    geo = lbm_amd.geo_poiseuille(nx, ny, nz)
    plan = ldist.slab_plan(nz, world)
    z0, z1 = plan[rank]
    sg = cases.slab_geo(geo, z0, z1)
    # the id rank 0 makes reaches every rank unchanged
    uid = ldist.share_unique_id(rank, None, lambda: bytes(range(128)))
    # halo planes: my ghost planes must equal my neighbours' edge planes
    tops = [torch.zeros(ny * nx, dtype=torch.int8) for _ in range(world)]
    bots = [torch.zeros(ny * nx, dtype=torch.int8) for _ in range(world)]
    dist.all_gather(tops, torch.from_numpy(sg[-2].reshape(-1).copy()))
    dist.all_gather(bots, torch.from_numpy(sg[1].reshape(-1).copy()))
    ok_halo = True
    if rank > 0:
        ok_halo &= bool(np.array_equal(sg[0].reshape(-1), tops[rank - 1].numpy()))
    if rank + 1 < world:
        ok_halo &= bool(np.array_equal(sg[-1].reshape(-1), bots[rank + 1].numpy()))
    mx = ldist.max_over_ranks([rank + 0.5, -rank], None)
    sm = ldist.sum_over_ranks([float(((sg[1:-1]) == 4).sum())], None)
    xa = lbm_amd.x_align_for(geo, lbm_amd.LBM_CASE_POISEUILLE)
    xas = ldist.max_over_ranks([xa, -xa], None)
    dist.barrier()
    np.save(os.path.join(out_dir, f"r{rank}.npy"), np.array(
        [z0, z1, uid == bytes(range(128)), ok_halo, mx[0], mx[1], sm[0], int((geo == 4).sum()), xas[0], -xas[1]],
        dtype=np.float64))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_slab_coordination(tmp_path, world):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    rows = [np.load(tmp_path / f"r{r}.npy") for r in range(world)]
    bounds = [(int(r[0]), int(r[1])) for r in rows]
    assert bounds[0][0] == 0 and bounds[-1][1] == 23
    assert all(bounds[i][1] == bounds[i + 1][0] for i in range(world - 1))
    for r in rows:
        assert r[2] == 1 and r[3] == 1            # id delivered; halo planes consistent
        assert r[4] == world - 0.5 and r[5] == 0  # max over ranks
        assert r[6] == r[7]                       # slabs' fluid cells add up to the lattice's
        assert r[8] == r[9]                       # every rank derives the same row alignment


def test_slab_plan_edges():
    import lbm_amd.dist as ldist
    assert ldist.slab_plan(512 * 8, 8)[3] == (1536, 2048)
    assert ldist.slab_plan(10, 3) == [(0, 4), (4, 7), (7, 10)]
    with pytest.raises(ValueError):
        ldist.slab_plan(2, 3)
