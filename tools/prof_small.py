#!/usr/bin/env python3
"""Launch-bound configurations for profiling: LDC 64^3 (the reference's published config),
Poiseuille 128x512x128 (C3) and the shipped bifurcation (C4), each stepped `steps` times
after a warm-up, wall time per step printed per case.
    rocprofv3 --kernel-trace --stats --output-format csv -d <dir> -- python3 tools/prof_small.py 500
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: E402,F401
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 500
which = sys.argv[2].split(",") if len(sys.argv) > 2 else ["ldc64", "c3", "c4"]


def run(name, lat, cells):
    lat.step(20, history=False)
    lat.sync()
    t = time.perf_counter()
    lat.step(steps, history=False)
    lat.sync()
    dt = time.perf_counter() - t
    # the k_step launches alone (HIP events around each; a separate, shorter pass)
    lat.profile(True)
    lat.step(min(steps, 200), history=False)
    st = lat.stats()
    lat.close()
    kus = st["step_kernel_ms"] / max(1, st["step_kernel_launches"]) * 1e3
    print(f"{name}: {dt / steps * 1e6:.2f} us/step, {cells * steps / dt / 1e6:.1f} MLUPS ({cells} cells); "
          f"k_step {kus:.2f} us", flush=True)


for w in which:
    if w.startswith("ldc"):
        n = int(w[3:])
        run(f"LDC {n}^3", cases.ldc_device(n, n, n), n ** 3)
    elif w == "c3":
        lat, geo = cases.poiseuille(128, 512, 128)
        run("Poiseuille 128x512x128 (NLATTICE)", lat, lbm_amd.index_transform(geo)[0])
    elif w == "c4":
        lat, geo, _, _ = cases.bifurcation(1)
        run("bifurcation 64x83x32 (NLATTICE)", lat, lbm_amd.index_transform(geo)[0])
