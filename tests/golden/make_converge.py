#!/usr/bin/env python3
"""Regenerate tests/golden/converge.json: the reference's default loops run to convergence
by the CPU oracle -- LDC 64^3 (config C1, ldc.cu:612-691, race-free two-phase wall order) and
Poiseuille 64^3 (Poiseulle.cu:940-1030) -- once with thrust's fp32 |u| sum emulated serially
in the reference storage order (the survey's emulation numbers: 5711 and 6230) and once with
the fp32 |u| terms summed in fp64, which is what liblbm does.  For the fp64 run the stop step,
the last residual and the SHA-256 of the fluid (rho, ux, uy, uz) bits at that step are kept:
the GPU test (test_gpu_converge.py) must stop at the same step with the same field bits.

    python tests/golden/make_converge.py      # ~5 min on one core per case
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
import orc  # noqa: E402


def sha_fluid(o, fluid):
    h = hashlib.sha256()
    for a in o.macros():
        h.update(np.ascontiguousarray(a[fluid]).tobytes())
    return h.hexdigest()


def run(name, kind, geo, tau, kw, fluid_code):
    out = {"shape_zyx": list(geo.shape), "tau": tau, "loop": "max_it 10000, stag_max 50, tol 1e-6"}
    for mode in ("fp32_serial", "fp64"):
        o = orc.Oracle(kind, geo, tau, **kw)
        o.residual_fp64(mode == "fp64")
        t = time.time()
        k, res = o.run_converge(10000, 50, 1e-6)
        out[f"stop_k_{mode}"] = int(k)
        out[f"residual_{mode}"] = res
        if mode == "fp64":
            fl = geo == fluid_code
            out["sha256_macros_fluid_fp64_stop"] = sha_fluid(o, fl)
            _, ux, uy, uz = o.macros()
            out["umax_fp64_stop"] = float(np.sqrt(ux[fl] ** 2 + uy[fl] ** 2 + uz[fl] ** 2).max())
            out["uy_max_fp64_stop"] = float(uy[fl].max())
        print(f"{name} {mode}: k={k} residual={res:.3e} ({time.time() - t:.0f} s)", flush=True)
    return out


def main():
    import lbm_amd
    res = {}
    res["ldc64_two_phase"] = run("ldc64", orc.LDC, orc.geo_ldc(64, 64, 64), 0.55, {"ldc_order": orc.TWO_PHASE}, 3)
    g = orc.geo_poiseuille(64, 64, 64)
    prof = lbm_amd.poiseuille_profile(64, 64)
    res["poiseuille64"] = run("pois64", orc.POISEUILLE, g, 0.58, {"inlet_uy": prof, "outlet_uy": prof}, 4)
    with open(os.path.join(HERE, "converge.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
