#!/usr/bin/env python3
"""Sparse lattices on the 4-cell path (C4 x4 upsampled, the synthetic coronary tree, C3) with
the liblbm.so LBM_LIBRARY names, for interleaved A/B runs of library variants.
    LBM_LIBRARY=<dir>/liblbm.so python3 tools/lab_sparse.py <tag>"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: E402,F401
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
for name in ("c4x4", "coronary", "c3"):
    if name == "c4x4":
        lat, raw = cases.bifurcation_upsampled(4)
        nl = lbm_amd.index_transform(lat.geo())[0]
        steps = 200
    elif name == "coronary":
        lat, geo = cases.coronary(cases.coronary_reference_vessel())
        nl = lbm_amd.index_transform(geo)[0]
        steps = 500
    else:
        lat, geo = cases.poiseuille(128, 512, 128)
        nl = lbm_amd.index_transform(geo)[0]
        steps = 200
    lat.step(20, history=False)
    lat.sync()
    t = time.perf_counter()
    lat.step(steps, history=False)
    lat.sync()
    dt = time.perf_counter() - t
    print(f"{tag} {name}: {nl * steps / dt / 1e6:.0f} NLATTICE-MLUPS {dt / steps * 1e6:.1f} us/step", flush=True)
    lat.close()
