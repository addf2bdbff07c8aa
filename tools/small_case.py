#!/usr/bin/env python3
"""Step a small LDC cavity (default 64^3, the reference's published config) for profiling:
    rocprofv3 --kernel-trace --output-format csv -d <dir> -- python3 tools/small_case.py 64 200"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: E402,F401
from lbm_amd import cases  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
lat = cases.ldc_device(n, n, n)
lat.step(20, history=False)
lat.sync()
t = time.perf_counter()
lat.step(steps, history=False)
lat.sync()
dt = time.perf_counter() - t
print(f"LDC {n}^3: {n ** 3 * steps / dt / 1e6:.1f} MLUPS, {dt / steps * 1e6:.2f} us/step")
