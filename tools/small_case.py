#!/usr/bin/env python3
"""Step a small LDC cavity (default 64^3, the reference's published config) for profiling:
    rocprofv3 --kernel-trace --output-format csv -d <dir> -- python3 tools/small_case.py 64 200
A third argument 'slab' builds the cube as the middle z-slab of a 3-slab cavity and attaches a
one-rank RCCL communicator: the multi-GPU step sequence (edge planes, interior, residual
all-reduce, finisher) without peers -- the per-GPU cost of the N > 1 bench minus the halo."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: E402,F401
from lbm_amd import cases  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
slab = len(sys.argv) > 3 and sys.argv[3] == "slab"
if slab:
    import lbm_amd  # noqa: E402
    lat = cases.ldc_device(n, n, n, z_offset=n, nz_global=3 * n)
    lat.attach_rccl(lbm_amd.rccl_unique_id(), 0, 1)
else:
    lat = cases.ldc_device(n, n, n)
lat.step(20, history=False)
lat.sync()
t = time.perf_counter()
lat.step(steps, history=False)
lat.sync()
dt = time.perf_counter() - t
print(f"LDC {n}^3{' slab+rccl' if slab else ''}: {n ** 3 * steps / dt / 1e6:.1f} MLUPS, {dt / steps * 1e6:.2f} us/step")
