#!/usr/bin/env python3
"""C3's two speeds: fresh C3 lattices in one process, each timed
with per-launch HIP events split by source buffer, beside its placement (candidates' write rates,
the two kept) and the device addresses of its buffers (lab build tools/lab_build.py ptrs).

    LBM_LIBRARY=tools/ab/ptrs/liblbm.so python3 tools/c3_modes_lab.py [lattices] [steps]
"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: F401,E402
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
for i in range(n):
    lat = cases.poiseuille(128, 512, 128)[0]
    ptr = (C.c_ulonglong * 6)()
    assert lbm_amd.lbm_lib().lbm_lab_ptrs(lat.h, ptr) == 0
    lat.step(20, history=False)
    lat.sync()
    lat.profile(1)
    lat.step(steps, history=False)
    lat.sync()
    st = lat.stats()
    pl = lat.placement()
    lat.close()
    kept = [pl["candidate_write_gbs"][k] for k in pl["chosen"]] if pl["candidate_write_gbs"] else []
    rec = {"i": i, "step_us": round(st["step_kernel_ms"] / max(1, st["step_kernel_launches"]) * 1e3, 2),
           "src0_us": round(st["step_kernel_src0_ms"] / max(1, st["step_kernel_src0_launches"]) * 1e3, 2),
           "src1_us": round(st["step_kernel_src1_ms"] / max(1, st["step_kernel_src1_launches"]) * 1e3, 2),
           "kept_gbs": kept, "best_gbs": max(pl["candidate_write_gbs"], default=None),
           "alloc0": hex(ptr[0]), "alloc1": hex(ptr[1]), "d01_mib": round((ptr[1] - ptr[0]) / 2**20, 3),
           "type": hex(ptr[2]), "chunks": hex(ptr[3]), "cells": hex(ptr[4])}
    print(json.dumps(rec), flush=True)
