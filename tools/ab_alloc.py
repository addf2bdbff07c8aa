#!/usr/bin/env python3
"""A/B of the population-buffer placement: per source buffer average k_step duration (HIP
events) next to the candidates' sweep-write rates, interleaved rounds so box drift hits every
variant; each round builds a fresh lattice, so every variant sees new allocations.

    python tools/ab_alloc.py ROUNDS VARIANT [VARIANT ...]
VARIANT = LBM_TUNE_BUFFER_ALLOC value: 0 (default) probe up to six candidates and keep the two
fastest-writing, 1 the first two allocations.  AB_CASES (default "ldc512"): comma-separated
ldcN (device cavity N^3) and c3 (Poiseuille 128 x 512 x 128, pipe along y).
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
which = os.environ.get("AB_CASES", "ldc" + os.environ.get("AB_N", "512")).split(",")


def make(w):
    if w == "c3":
        return cases.poiseuille(128, 512, 128)[0], 100
    n = int(w[3:])
    return cases.ldc_device(n, n, n), 20 if n >= 512 else 100


for r in range(rounds):
    for w in which:
        for v in variants:
            with lbm_amd.tuned(lbm_amd.TUNE_BUFFER_ALLOC, int(v)):
                lat, steps = make(w)
            lat.step(6, history=False)
            lat.sync()
            lat.profile(True)
            lat.step(steps, history=False)
            lat.sync()
            st = lat.stats()
            pl = lat.placement()
            lat.close()
            out = {"round": r, "case": w, "variant": v,
                   "src0_us": round(st["step_kernel_src0_ms"] / st["step_kernel_src0_launches"] * 1e3, 2),
                   "src1_us": round(st["step_kernel_src1_ms"] / st["step_kernel_src1_launches"] * 1e3, 2),
                   "avg_us": round(st["step_kernel_ms"] / st["step_kernel_launches"] * 1e3, 2), **pl}
            print(json.dumps(out), flush=True)
