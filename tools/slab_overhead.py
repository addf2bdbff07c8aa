#!/usr/bin/env python3
"""Per-GPU cost of the multi-GPU step sequence at C5's per-GPU size: LDC 512^3 as one domain
against the same 512^3 as the middle z-slab of a 512 x 512 x 1536 cavity with a one-rank RCCL
communicator (edge-plane launch, interior launch, slab reduction, all-reduce and finisher on
the communication stream; no peers, so no halo bytes).  Interleaved rounds, wall ms per step.
    python3 tools/slab_overhead.py [steps] [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: E402,F401
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n = 512
for r in range(rounds):
    for mode in ("single", "slab+rccl"):
        if mode == "single":
            lat = cases.ldc_device(n, n, n)
        else:
            lat = cases.ldc_device(n, n, n, z_offset=n, nz_global=3 * n)
            lat.attach_rccl(lbm_amd.rccl_unique_id(), 0, 1)
        lat.step(5, history=False)
        lat.sync()
        lat.profile(True)
        t = time.perf_counter()
        lat.step(steps, history=False)
        lat.sync()
        dt = time.perf_counter() - t
        st = lat.stats()
        lat.close()
        extra = ""
        if mode != "single":
            extra = (f" edge {st['edge_ms'] / steps:.4f} interior {st['interior_ms'] / steps:.4f}"
                     f" (ms/step, HIP events)")
        print(f"round {r} {mode}: {dt / steps * 1e3:.4f} ms/step, {n ** 3 * steps / dt / 1e6:.0f} MLUPS{extra}",
              flush=True)
