#!/usr/bin/env python3
"""Sweep of the layout / path knobs on the latency-bound lattices (LDC 64^3, bifurcation C4):
row axis (x, y) x cells per lane (1, 4), interleaved rounds, wall us/step.
    python3 tools/lab_small_knobs.py [steps] [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: E402,F401
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for r in range(rounds):
    for name in ("ldc64", "c4"):
        for axis in (1, 2):
            for cpl in (1, 4):
                lbm_amd.tune(lbm_amd.TUNE_ROW_AXIS, axis)
                lbm_amd.tune(lbm_amd.TUNE_CELLS_PER_LANE, cpl)
                if name == "ldc64":
                    lat, geo = cases.ldc(64)
                    cells = 64 ** 3
                else:
                    lat, geo, _, _ = cases.bifurcation(1)
                    cells = lbm_amd.index_transform(geo)[0]
                lat.step(50, history=False)
                lat.sync()
                t = time.perf_counter()
                lat.step(steps, history=False)
                lat.sync()
                dt = time.perf_counter() - t
                lay = lat.layout()
                print(f"round {r} {name} rows={'xy'[axis - 1]} cells/lane={cpl} chunks={lay['active_chunks']}: "
                      f"{dt / steps * 1e6:.2f} us/step {cells * steps / dt / 1e6:.0f} MLUPS", flush=True)
                lat.close()
