#!/usr/bin/env python3
"""Fixed cost per launch: k_step time of the pipe and the cavity at growing lengths (measurement
tool).  A launch costs t = t0 + cells / rate; t0 (ramp-up of the first round of waves and the
tail of the last) is what a lattice of few rounds, like C3's 12, pays on top of the streaming
rate.  Pipe 128 x L x 128 (C3 is L = 512) and cavity 512 x 512 x Z, both four cells per lane.

    python3 tools/scale_lab.py [rounds]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: F401,E402
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402


def kstep_us(lat, steps):
    nf = lat.counts()["n_fluid"]
    lat.step(10, history=False)
    lat.sync()
    lat.profile(True)
    lat.step(steps, history=False)
    lat.sync()
    st = lat.stats()
    shape = lat.launch_shape()
    lat.close()
    return st["step_kernel_ms"] / st["step_kernel_launches"] * 1e3, nf, shape["main_blocks"]


for kv in filter(None, os.environ.get("AB_TUNE", "").split(",")):  # "knob:value,...": lbm_tune
    k, v = kv.split(":")
    lbm_amd.tune(int(k), int(v))
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
only = os.environ.get("SCALE_ONLY", "")
for r in range(rounds):
    for L in (256, 512, 1024, 2048) if only != "ldc" else ():
        us, nf, mb = kstep_us(cases.poiseuille(128, L, 128)[0], 100)
        print(json.dumps({"round": r, "lattice": f"pipe 128x{L}x128", "k_step_us": round(us, 2), "n_fluid": nf,
                          "chunk_blocks": mb, "ns_per_kcell": round(us * 1e6 / nf, 3)}), flush=True)
    for Z in (32, 64, 128, 256) if only != "pipe" else ():
        us, nf, mb = kstep_us(cases.ldc_device(512, 512, Z), 50)
        print(json.dumps({"round": r, "lattice": f"ldc 512x512x{Z}", "k_step_us": round(us, 2), "n_fluid": nf,
                          "chunk_blocks": mb, "ns_per_kcell": round(us * 1e6 / nf, 3)}), flush=True)
