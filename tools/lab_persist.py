#!/usr/bin/env python3
"""A/B of the persistent multi-step path (k_persist) against one k_step1 launch per step on the
latency-bound lattices (LDC 32^3 / 64^3, bifurcation C4), interleaved rounds, wall us/step.
    python3 tools/lab_persist.py [steps] [rounds]"""
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
    for name in ("ldc32", "ldc64", "c4"):
        for pers in (1, 0, 2, 3):
            lbm_amd.tune(lbm_amd.TUNE_PERSISTENT, pers)
            if name.startswith("ldc"):
                n = int(name[3:])
                lat = cases.ldc_device(n, n, n)
                cells = n ** 3
            else:
                lat, geo, _, _ = cases.bifurcation(1)
                cells = lbm_amd.index_transform(geo)[0]
            lat.step(50, history=False)
            lat.sync()
            t = time.perf_counter()
            lat.step(steps, history=False)
            lat.sync()
            dt = time.perf_counter() - t
            path, wg = lat.step_path()
            print(f"round {r} {name} path={path} wg={wg}: {dt / steps * 1e6:.2f} us/step "
                  f"{cells * steps / dt / 1e6:.0f} MLUPS", flush=True)
            lat.close()
