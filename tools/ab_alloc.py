#!/usr/bin/env python3
"""A/B of the population-buffer placement at LDC 512^3: per source buffer average k_step
duration (HIP events), interleaved rounds so box drift hits every variant; each round builds a
fresh lattice, so every variant sees new allocations.

    python tools/ab_alloc.py ROUNDS VARIANT [VARIANT ...]
VARIANT = LBM_TUNE_BUFFER_ALLOC value: 0 (default) probe up to six candidates and keep the two
fastest-writing, 1 the first two allocations.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: F401,E402
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
variants = sys.argv[2:] or ["0", "1"]
n = int(os.environ.get("AB_N", "512"))
for r in range(rounds):
    for v in variants:
        with lbm_amd.tuned(lbm_amd.TUNE_BUFFER_ALLOC, int(v)):
            lat = cases.ldc_device(n, n, n)
        lat.step(6, history=False)
        lat.sync()
        lat.profile(True)
        lat.step(20, history=False)
        lat.sync()
        st = lat.stats()
        pl = lat.placement()
        lat.close()
        out = {"round": r, "variant": v,
               "src0_ms": round(st["step_kernel_src0_ms"] / st["step_kernel_src0_launches"], 4),
               "src1_ms": round(st["step_kernel_src1_ms"] / st["step_kernel_src1_launches"], 4),
               "avg_ms": round(st["step_kernel_ms"] / st["step_kernel_launches"], 4), **pl}
        print(json.dumps(out), flush=True)
