#!/usr/bin/env python3
"""Short LDC n^3 run for rocprofv3 counter passes: K launches of the chosen step kernel
(LBM_TUNE_STEPS_PER_LAUNCH = argv[2], default 2)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: F401,E402
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
lbm_amd.tune(lbm_amd.TUNE_STEPS_PER_LAUNCH, k)
lat = cases.ldc_device(n, n, n)
lat.step(steps, history=False)
lat.sync()
lat.close()
print("done")
