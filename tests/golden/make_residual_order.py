#!/usr/bin/env python3
"""Regenerate tests/golden/residual_order.json: where the reference's default loops stop when
the per-step |u| sum S is formed the way thrust::reduce forms it on a CUDA GPU.

The reference sums S in fp32 with thrust::reduce (ldc.cu:460-466, 660-662; Poiseulle.cu:895-901,
993-1002), i.e. CUB's two-pass device reduction.  Its tree shape depends on the CUB / thrust
version and the GPU (tuning policy: items per thread, vector width; grid cap = SM count x blocks
per SM x subscription factor), none of which the reference records.  So the CPU oracle runs
LDC 64^3 (config C1, two-phase wall order) and Poiseuille 64^3 to convergence under several
plausible parameter sets of the CUB tree (oracle/lbm_oracle.c orc_cub_reduce), next to the serial
fp32 sum and liblbm's fp64 sum (tests/golden/converge.json).  For each run: the stop step, the
last residual and the SHA-256 of the fluid (rho, u) bits at the stop.

    python tests/golden/make_residual_order.py      # ~10 min on 6 cores
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))

# (items per thread, vector load width, grid cap): CUB DeviceReduce's sm_60+ policy (256 threads,
# 16 items of 4 B, vector 4) and thrust's own reduce tunings (20 items, vector 4 / 2), on a
# 6-SM GTX 1050 Ti (thesis 4.9.1) at 8 blocks per SM x subscription factor 5 = 240 blocks, or at
# one block per SM (30)
PARAMS = {
    "cub_i16_v4_g240": (16, 4, 240),
    "thrust_i20_v4_g240": (20, 4, 240),
    "thrust_i20_v2_g240": (20, 2, 240),
    "cub_i16_v4_g30": (16, 4, 30),
}


def sha_fluid(o, fluid):
    h = hashlib.sha256()
    for a in o.macros():
        h.update(np.ascontiguousarray(a[fluid]).tobytes())
    return h.hexdigest()


def one(args):
    case, pname = args
    os.environ["OMP_NUM_THREADS"] = "1"
    import orc
    import lbm_amd
    if case == "ldc64_two_phase":
        geo, kind, tau, kw, fc = orc.geo_ldc(64, 64, 64), orc.LDC, 0.55, {"ldc_order": orc.TWO_PHASE}, 3
    else:
        geo = orc.geo_poiseuille(64, 64, 64)
        prof = lbm_amd.poiseuille_profile(64, 64)
        kind, tau, kw, fc = orc.POISEUILLE, 0.58, {"inlet_uy": prof, "outlet_uy": prof}, 4
    o = orc.Oracle(kind, geo, tau, **kw)
    o.residual_cub_tree(*PARAMS[pname])
    t = time.time()
    k, res = o.run_converge(10000, 50, 1e-6)
    out = {"params_ipt_vec_grid": list(PARAMS[pname]), "stop_k": int(k), "residual": res,
           "sha256_macros_fluid_stop": sha_fluid(o, geo == fc), "seconds": round(time.time() - t, 1)}
    print(f"{case} {pname}: k={k} ({out['seconds']} s)", flush=True)
    return case, pname, out


def main():
    jobs = [(c, p) for c in ("ldc64_two_phase", "poiseuille64") for p in PARAMS]
    res = {c: {} for c in ("ldc64_two_phase", "poiseuille64")}
    with ProcessPoolExecutor(max_workers=min(6, len(jobs))) as ex:
        for case, pname, out in ex.map(one, jobs):
            res[case][pname] = out
    with open(os.path.join(HERE, "converge.json")) as f:
        conv = json.load(f)
    for case in res:
        res[case]["serial_fp32"] = {"stop_k": conv[case]["stop_k_fp32_serial"]}
        res[case]["fp64_liblbm"] = {"stop_k": conv[case]["stop_k_fp64"]}
    with open(os.path.join(HERE, "residual_order.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
