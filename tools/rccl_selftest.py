#!/usr/bin/env python3
"""Two ranks exercising lbm_attach_rccl / the RCCL step path (halo exchange + residual
all-reduce) against a single-domain run.  Ranks use devices 0 and 1 when two are visible;
on a one-GPU box both use device 0, which RCCL refuses (ncclCommInitRank: invalid usage,
observed on MI355X / RCCL 2.26.6) -- the script then reports that and exits 0."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))


def worker(rank, world, port, out):
    import torch  # noqa: F401  shared HIP runtime
    import torch.distributed as dist
    import lbm_amd
    from lbm_amd import cases
    from lbm_amd import dist as ldist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    n, nzl = 32, 16
    dev = rank if torch.cuda.device_count() >= world else 0
    lat = cases.ldc_device(n, n, nzl, z_offset=rank * nzl, nz_global=nzl * world, device=dev)
    try:
        lat.attach_rccl(ldist.share_unique_id(rank, None, lbm_amd.rccl_unique_id), rank, world)
    except Exception as e:  # noqa: BLE001
        np.save(os.path.join(out, f"err{rank}.npy"), np.array([str(e)]))
        dist.destroy_process_group()
        return
    hist = lat.step(40)
    rho, ux, uy, uz = lat.macros()
    np.savez(os.path.join(out, f"r{rank}.npz"), hist=hist, ux=ux, uy=uy, uz=uz)
    lat.close()
    dist.barrier()
    dist.destroy_process_group()


def main():
    import tempfile
    out = tempfile.mkdtemp(dir=os.path.join(REPO, "gpurun_out") if os.path.isdir(os.path.join(REPO, "gpurun_out")) else None)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    mp.start_processes(worker, args=(world, port, out), nprocs=world, join=True, start_method="spawn")
    errs = [f for f in os.listdir(out) if f.startswith("err")]
    if errs:
        print("RCCL refused:", np.load(os.path.join(out, errs[0]))[0])
        return 0
    import torch  # noqa: F401
    import lbm_amd  # noqa: F401
    from lbm_amd import cases
    one = cases.ldc_device(32, 32, 32, device=0)
    h1 = one.step(40)
    ref = one.macros()
    ok = True
    for r in range(world):
        d = np.load(os.path.join(out, f"r{r}.npz"))
        for k, a in zip(("ux", "uy", "uz"), ref[1:]):
            same = np.array_equal(d[k].view(np.uint32), a[r * 16:(r + 1) * 16].view(np.uint32))
            ok &= same
            print(f"rank {r} {k}: {'bitwise' if same else 'DIFFERS'}")
        print(f"rank {r} residual max |diff| {np.abs(d['hist'] - h1).max():.3e}")
    print("RCCL two-rank slab run", "OK" if ok else "MISMATCH")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
