#!/usr/bin/env python3
"""A/B of the population-buffer placement at LDC 512^3: per source buffer average k_step
duration (HIP events), interleaved rounds so box drift hits every variant.

    python tools/ab_alloc.py ROUNDS VARIANT [VARIANT ...]
VARIANT = MODE[:GAP_KB] (LBM_TUNE_BUFFER_ALLOC, LBM_TUNE_BUFFER_GAP_KB), e.g. 0 2 1:0 1:4 1:1024
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
variants = sys.argv[2:] or ["0", "1:0", "2"]
n = int(os.environ.get("AB_N", "512"))
for r in range(rounds):
    for v in variants:
        mode, _, gap = v.partition(":")
        with lbm_amd.tuned(lbm_amd.TUNE_BUFFER_ALLOC, int(mode)), lbm_amd.tuned(lbm_amd.TUNE_BUFFER_GAP_KB,
                                                                                int(gap or 0)):
            lat = cases.ldc_device(n, n, n)
        lat.step(6, history=False)
        lat.sync()
        lat.profile(True)
        lat.step(20, history=False)
        lat.sync()
        st = lat.stats()
        lat.close()
        out = {"round": r, "variant": v,
               "src0_ms": round(st["step_kernel_src0_ms"] / st["step_kernel_src0_launches"], 4),
               "src1_ms": round(st["step_kernel_src1_ms"] / st["step_kernel_src1_launches"], 4),
               "avg_ms": round(st["step_kernel_ms"] / st["step_kernel_launches"], 4)}
        print(json.dumps(out), flush=True)
