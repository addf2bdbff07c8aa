#!/usr/bin/env python3
"""Regenerate tests/golden/golden.json + golden.npz: oracle outputs on small inputs.

The inputs are the reference's own set-ups (geo_pre boxes, the Poiseuille pipe with its
`uygt` inlet/outlet, the shipped bifurcation geo.txt / bc.txt in this directory), so these
files are input -> expected-output vectors for the hot path.  They are produced by the CPU
oracle (oracle/lbm_oracle.c), whose pinning is described in oracle/PINNING.md; the tests
use them to
  * catch any drift of the oracle itself (test_golden.py, CPU), and
  * give the GPU path a fixed target independent of the oracle build (test_gpu_parity.py).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import orc  # noqa: E402

BIF = os.path.join(HERE, "bifurcation")
FLUID = {orc.LDC: 3, orc.POISEUILLE: 4, orc.MASK: 4}


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def case_setups():
    """name -> (kind, geo, tau, oracle kwargs, steps)."""
    out = {}
    out["ldc16_two_phase"] = (orc.LDC, orc.geo_ldc(16, 16, 16), 0.55, {"ldc_order": orc.TWO_PHASE}, 25)
    out["ldc16_serial"] = (orc.LDC, orc.geo_ldc(16, 16, 16), 0.55, {"ldc_order": orc.SERIAL_EMU}, 25)
    g = orc.geo_poiseuille(20, 24, 20)
    out["poiseuille_20x24x20"] = (orc.POISEUILLE, g, 0.58, {}, 40)
    raw = orc.read_geo_txt(os.path.join(BIF, "geo.txt"), 64, 83, 32)
    gb = orc.geo_mask(raw)
    _, inl, outl = orc.read_bc_txt(os.path.join(BIF, "bc.txt"), gb, 1)
    out["bif_inlet_block1"] = (orc.MASK, gb, 0.55, {"inlet_uy": inl, "outlet_uy": outl}, 100)
    return out


def poiseuille_tables(nx: int, nz: int):
    """uygt of Poiseulle.cu:329-352 (u_max = 0.09714700668), x fastest."""
    import lbm_amd  # host ingest library -- only for the inlet table shared by both sides
    return lbm_amd.poiseuille_profile(nx, nz)


def run(name, kind, geo, tau, kw, steps):
    if kind == orc.POISEUILLE:
        prof = poiseuille_tables(geo.shape[2], geo.shape[0])
        kw = dict(kw, inlet_uy=prof, outlet_uy=prof)
    o = orc.Oracle(kind, geo, tau, **kw)
    hist = o.step(steps)
    rho, ux, uy, uz = o.macros()
    fl = geo == FLUID[kind]
    f = o.f()
    return {
        "kind": kind, "shape_zyx": list(geo.shape), "tau": tau, "steps": steps,
        "oracle_kwargs": {k: v for k, v in kw.items() if not isinstance(v, np.ndarray)},
        "sha256_macros_fluid": sha(rho[fl], ux[fl], uy[fl], uz[fl]),
        "sha256_f_fluid": sha(f[:, fl]),
        "sha256_residuals": sha(hist),
        "umax": float(np.sqrt(ux[fl] ** 2 + uy[fl] ** 2 + uz[fl] ** 2).max()),
        "rho_min": float(rho[fl].min()), "rho_max": float(rho[fl].max()),
        "n_fluid": int(fl.sum()), "bad_reads": o.bad_reads(),
    }, (rho, ux, uy, uz, hist)


def main():
    sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
    meta, arrays = {}, {}
    for name, (kind, geo, tau, kw, steps) in case_setups().items():
        m, (rho, ux, uy, uz, hist) = run(name, kind, geo, tau, kw, steps)
        meta[name] = m
        if geo.size <= 16 ** 3:  # small enough to keep whole
            for k, a in zip(("rho", "ux", "uy", "uz"), (rho, ux, uy, uz)):
                arrays[f"{name}.{k}"] = a
            arrays[f"{name}.residuals"] = hist
        print(name, m["umax"], m["sha256_macros_fluid"][:16])
    json.dump(meta, open(os.path.join(HERE, "golden.json"), "w"), indent=1, sort_keys=True)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)


if __name__ == "__main__":
    main()
