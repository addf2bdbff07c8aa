#!/usr/bin/env python3
"""A/B of LBM_TUNE_GRID_STRIDE (1: one chunk per wave; 0: by sparsity; B >= 2: at most B blocks
per CU looping over their XCD's chunks) on the 4-cell lattices; interleaved rounds, MLUPS from the host clock."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: E402,F401
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

VALUES = [int(v) for v in os.environ.get("LAB_STRIDE", "1,0").split(",")]  # 1 off, 0 auto


def build(name):
    if name == "c3":
        lat, geo = cases.poiseuille(128, 512, 128)
        return lat, geo.size, 200
    if name == "c4x4":
        lat, raw = cases.bifurcation_upsampled(4)
        return lat, raw.size, 200
    if name == "coronary":
        lat, geo = cases.coronary(cases.coronary_reference_vessel())
        return lat, geo.size, 1000
    n = int(name[3:])
    return cases.ldc_device(n, n, n), n ** 3, 200 if n == 256 else 60


# bitwise check first: 4-cell LDC 128^3 and C4 x4 (lane masks), 30 steps, stride vs one chunk per wave
import numpy as np  # noqa: E402
for name in ("ldc128", "c4x4"):
    outs = []
    for v in (1, 2):
        with lbm_amd.tuned(lbm_amd.TUNE_CELLS_PER_LANE, 4), lbm_amd.tuned(lbm_amd.TUNE_GRID_STRIDE, v):
            lat = cases.ldc_device(128, 128, 128) if name == "ldc128" else cases.bifurcation_upsampled(4)[0]
        lat.step(30, history=False)
        outs.append(lat.f())
        lat.close()
    same = np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    print(f"bitwise {name}: {'equal' if same else 'DIFFERENT'}", flush=True)
    assert same

for rnd in range(3):
    for name in ("ldc512", "c3", "c4x4", "coronary"):
        for v in VALUES:
            with lbm_amd.tuned(lbm_amd.TUNE_GRID_STRIDE, v):
                lat, cells, steps = build(name)
            lat.step(20, history=False)
            lat.sync()
            t = time.perf_counter()
            lat.step(steps, history=False)
            lat.sync()
            dt = time.perf_counter() - t
            lat.close()
            print(f"round {rnd} {name} stride={v}: {cells * steps / dt / 1e6:.0f} MLUPS", flush=True)
