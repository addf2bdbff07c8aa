#!/usr/bin/env python3
"""A/B of one vs two time steps per launch (LBM_TUNE_STEPS_PER_LAUNCH) on LDC n^3: ms per
time step from HIP events around the step kernels, interleaved rounds.

    python tools/ab_steps.py [ROUNDS] [N] [STEPS]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: F401,E402
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
for r in range(rounds):
    for k in (1, 2):
        lbm_amd.tune(lbm_amd.TUNE_STEPS_PER_LAUNCH, k)
        lat = cases.ldc_device(n, n, n)
        lat.step(4, history=False)
        lat.sync()
        lat.profile(True)
        t = time.perf_counter()
        lat.step(steps, history=False)
        lat.sync()
        dt = time.perf_counter() - t
        st = lat.stats()
        lat.close()
        print(json.dumps({"round": r, "steps_per_launch": k, "n": n,
                          "kernel_ms_per_step": round(st["step_kernel_ms"] / steps, 4),
                          "wall_ms_per_step": round(dt / steps * 1e3, 4),
                          "mlups": round(n ** 3 * steps / dt / 1e6, 1),
                          "launches": st["step_kernel_launches"]}), flush=True)
