"""Pin the CPU oracle against every known answer available for the reference.

TEST INFRASTRUCTURE ONLY.  Writes oracle/pins.json; oracle/PINNING.md explains each
entry and its provenance.  Long-running (several minutes): the fast subset is
re-checked by tests/test_oracle_pins.py on every CPU test run.

Usage: python oracle/pin_check.py [--only NAME ...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import orc  # noqa: E402

REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden", "bifurcation")


def pin_poiseuille_converge():
    """SURVEY.md 3.2 [probe]: the unmodified Poiseulle.cu (64^3) stops at k = 6230 with
    uy_max = 0.096993; NLATTICE = 214128, 175200 fluid cells."""
    g = orc.geo_poiseuille(64, 64, 64)
    n, _ = orc.index_transform(g)
    o = orc.Oracle(orc.POISEUILLE, g, 0.58)
    t = time.time()
    k, res = o.run_converge()
    rho, ux, uy, uz = o.macros()
    fl = g == 4
    return {"nlattice": n, "fluid": int(fl.sum()), "stop_k": k, "last_residual": res,
            "uy_max": float(uy[fl].max()), "rho_min": float(rho[fl].min()), "rho_max": float(rho[fl].max()),
            "bad_reads": o.bad_reads(), "seconds": time.time() - t,
            "expect": {"nlattice": 214128, "fluid": 175200, "stop_k": 6230, "uy_max": 0.096993}}


def pin_ldc_serial_converge():
    """SURVEY.md 3.1 [probe]: the serial emulation of ldc.cu (64^3) stops at k = 5335."""
    g = orc.geo_ldc(64, 64, 64)
    o = orc.Oracle(orc.LDC, g, 0.55, ldc_order=orc.SERIAL_EMU)
    t = time.time()
    k, res = o.run_converge()
    rho, ux, uy, uz = o.macros()
    fl = g == 3
    return {"stop_k": k, "last_residual": res, "uz_max": float(uz[fl].max()), "uz_min": float(uz[fl].min()),
            "seconds": time.time() - t, "expect": {"stop_k": 5335}}


def pin_ldc_two_phase_converge():
    """Two-phase (race-free) LDC 64^3 to convergence: the build's LDC semantics. Reported
    beside the serial order; SURVEY.md App. B gives 2.0e-4 velocity rel-L2 between the two
    orders at 6000 steps."""
    g = orc.geo_ldc(64, 64, 64)
    a = orc.Oracle(orc.LDC, g, 0.55, ldc_order=orc.TWO_PHASE)
    b = orc.Oracle(orc.LDC, g, 0.55, ldc_order=orc.SERIAL_EMU)
    t = time.time()
    k, res = a.run_converge()
    b.step(k)
    fl = g == 3
    ua = np.stack(a.macros()[1:])[:, fl]
    ub = np.stack(b.macros()[1:])[:, fl]
    rel = float(np.linalg.norm(ua - ub) / np.linalg.norm(ub))
    return {"stop_k": k, "last_residual": res, "vel_relL2_two_phase_vs_serial_at_stop": rel,
            "seconds": time.time() - t}


def _bif(skip):
    raw = orc.read_geo_txt(os.path.join(GOLD, "geo.txt"), 64, 83, 32)
    g = orc.geo_mask(raw)
    nt, inl, out = orc.read_bc_txt(os.path.join(GOLD, "bc.txt"), g, skip)
    o = orc.Oracle(orc.MASK, g, 0.55, inlet_uy=inl, outlet_uy=out)
    t = time.time()
    o.step(4401)  # bifurcation.cu:1246, i = 0..REPEAT inclusive
    rho, ux, uy, uz = o.macros()
    fl = g == 4
    umag = np.sqrt(ux ** 2 + uy ** 2 + uz ** 2)[fl]
    return {"umax": float(umag.max()), "rho_min": float(rho[fl].min()), "rho_max": float(rho[fl].max()),
            "bad_reads": o.bad_reads(), "seconds": time.time() - t}


def pin_bif_as_shipped():
    """SURVEY.md 0.6 [probe]: as shipped, |u|max = 3.5e-6 after 4401 steps."""
    r = _bif(0)
    r["expect"] = {"umax": 3.5e-6}
    return r


def pin_bif_inlet_block1():
    """SURVEY.md 0.6 [probe]: with bc.txt block 1 as the inlet, |u|max 0.224, rho in [0.994, 1.141]."""
    r = _bif(1)
    r["expect"] = {"umax": 0.224, "rho_min": 0.994, "rho_max": 1.141}
    return r


def pin_geometry():
    """Known answers of the host ingest: thesis section 4.8 (NLATTICE 65820 for the bifurcation)
    and SURVEY.md 3.3 class counts; bc.txt token count (6144)."""
    raw = orc.read_geo_txt(os.path.join(GOLD, "geo.txt"), 64, 83, 32)
    g = orc.geo_mask(raw)
    n, _ = orc.index_transform(g)
    counts = {int(k): int(v) for k, v in zip(*np.unique(g, return_counts=True))}
    nt, _, _ = orc.read_bc_txt(os.path.join(GOLD, "bc.txt"), g, 1)
    gp = orc.geo_poiseuille(64, 64, 64)
    npz, _ = orc.index_transform(gp)
    return {"bif_nlattice": n, "bif_counts": counts, "bc_tokens": nt, "raw_zeros": int((raw == 0).sum()),
            "raw_ones": int((raw == 1).sum()), "poiseuille_nlattice": npz,
            "expect": {"bif_nlattice": 65820,
                       "bif_counts": {4: 45307, 1: 7648, 2: 345, 3: 306, -1: 12214, 0: 104164},
                       "bc_tokens": 6144, "raw_zeros": 115596, "raw_ones": 54388, "poiseuille_nlattice": 214128}}


PINS = {f.__name__[4:]: f for f in (pin_geometry, pin_bif_as_shipped, pin_bif_inlet_block1,
                                     pin_poiseuille_converge, pin_ldc_serial_converge,
                                     pin_ldc_two_phase_converge)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    path = os.path.join(HERE, "pins.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name, fn in PINS.items():
        if args.only and name not in args.only:
            continue
        print(f"[pin] {name} ...", flush=True)
        out[name] = fn()
        print(json.dumps(out[name]), flush=True)
        json.dump(out, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
