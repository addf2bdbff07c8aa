#!/usr/bin/env python3
"""MLUPS of the mid-size lattices (LDC 256^3 = C2, Poiseuille 128x512x128 = C3, LDC 512^3) with
the liblbm.so LBM_LIBRARY names, for interleaved A/B runs of library variants:
    for i in 1 2 3; do for v in a b; do LBM_LIBRARY=$v/liblbm.so python3 tools/lab_sizes.py $v; done; done"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: E402,F401
from lbm_amd import cases  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["ldc256", "c3", "ldc512"]
for name in names:
    if name == "c3":
        lat, geo = cases.poiseuille(128, 512, 128)
        cells, steps = geo.size, 200
    else:
        n = int(name[3:])
        lat = cases.ldc_device(n, n, n)
        cells, steps = n ** 3, 200 if n == 256 else int(os.environ.get("LAB_STEPS512", "50"))
    lat.step(20, history=False)
    lat.sync()
    t = time.perf_counter()
    lat.step(steps, history=False)
    lat.sync()
    dt = time.perf_counter() - t
    print(f"{tag} {name}: {cells * steps / dt / 1e6:.0f} MLUPS placement {lat.placement()}", flush=True)
    lat.close()
