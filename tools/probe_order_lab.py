#!/usr/bin/env python3
"""Does the streaming probe's allocation round (16 x 8 GiB, freed) change the placement
candidates a later lattice draws?  Alternating fresh processes: 'probe' runs
lbm_probe_stream_shapes first, 'plain' does not; both then build LDC 256^3 (C2) and report its
placement candidates and k_step time (measurement tool).

    python3 tools/probe_order_lab.py <rounds>
"""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode):
    sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
    import torch  # noqa: F401
    import lbm_amd
    from lbm_amd import cases
    if mode == "probe":
        lbm_amd.probe_stream_shapes(0)
    lat = cases.ldc_device(256, 256, 256)
    lat.step(20, history=False)
    lat.sync()
    lat.profile(True)
    t = time.perf_counter()
    lat.step(200, history=False)
    lat.sync()
    dt = time.perf_counter() - t
    st = lat.stats()
    out = {"mode": mode, "us_step": round(dt / 200 * 1e6, 2),
           "k_step_us": round(st["step_kernel_ms"] / max(1, st["step_kernel_launches"]) * 1e3, 2),
           "placement": lat.placement()}
    lat.close()
    print("PL " + json.dumps(out), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        sys.exit(0)
    for r in range(int(sys.argv[1])):
        for mode in ("probe", "plain"):
            p = subprocess.run([sys.executable, __file__, "--child", mode], capture_output=True, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("PL ")]
            print(line[0][3:] if line else f"{mode} round {r}: rc {p.returncode} {p.stderr[-800:]}", flush=True)
