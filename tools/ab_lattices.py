#!/usr/bin/env python3
"""Interleaved A/B of liblbm builds on the bench's secondary lattices (run through gpurun).

    python3 tools/ab_lattices.py <rounds> <variant> ...     # variant: product | a dir with liblbm.so,
                                                            # optionally "@knob:value,..." (lbm_tune)
    python3 tools/ab_lattices.py --child <cases>            # one process per (round, variant)

Each (round, variant) is a fresh process with LBM_LIBRARY pointing at the variant, so builds
alternate on one box and drift (clocks, thermals) hits all of them alike.  Per case: wall time
per step over `steps` steps after a warm-up, and k_step's mean launch time from HIP events.
"""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = "ldc64,c4,c3,c4x4,coronary,ldc256,ldc512"


def child(which):
    sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
    import torch  # noqa: F401
    import lbm_amd
    from lbm_amd import cases
    for kv in filter(None, os.environ.get("AB_TUNE", "").split(",")):  # "knob:value,...": lbm_tune
        k, v = kv.split(":")
        lbm_amd.tune(int(k), int(v))

    def run(lat, steps):
        shape = lat.launch_shape()
        place = lat.placement()
        nf = lat.counts()["n_fluid"]
        lat.step(20, history=False)
        lat.sync()
        t = time.perf_counter()
        lat.step(steps, history=False)
        lat.sync()
        dt = time.perf_counter() - t
        lat.profile(True)
        lat.step(min(steps, 200), history=False)
        st = lat.stats()
        lat.close()
        return {"us_step": round(dt / steps * 1e6, 2),
                "k_step_us": round(st["step_kernel_ms"] / max(1, st["step_kernel_launches"]) * 1e3, 2),
                "n_fluid": nf, "launch_shape": shape, "placement": place}

    out = {}
    for w in which.split(","):
        if w == "c5":  # the C5 lattice (512 x 512 x 4096, ~187 GB) as one domain
            out[w] = run(cases.ldc_device(512, 512, 4096), 10)
        elif w.startswith("ldc"):
            n = int(w[3:])
            out[w] = run(cases.ldc_device(n, n, n), 2000 if n <= 64 else 200 if n <= 256 else 30)
        elif w == "c3":
            out[w] = run(cases.poiseuille(128, 512, 128)[0], 300)
        elif w == "c4":
            out[w] = run(cases.bifurcation(1)[0], 2000)
        elif w == "c4x4":
            out[w] = run(cases.bifurcation_upsampled(4)[0], 300)
        elif w == "coronary":
            out[w] = run(cases.coronary(cases.coronary_reference_vessel())[0], 1000)
    out["kernel_src"] = lbm_amd.kernel_fingerprint()
    print("AB " + json.dumps(out), flush=True)


def main():
    rounds = int(sys.argv[1])
    variants = sys.argv[2:]
    which = os.environ.get("AB_CASES", CASES)
    res = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            env = dict(os.environ)
            lib, _, tune = v.partition("@")
            env["AB_TUNE"] = tune
            if lib == "product":
                env.pop("LBM_LIBRARY", None)
            else:
                env["LBM_LIBRARY"] = os.path.join(REPO, lib, "liblbm.so")
            p = subprocess.run([sys.executable, __file__, "--child", which], env=env, capture_output=True, text=True,
                               timeout=600)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("AB ")]
            if p.returncode != 0 or not line:
                print(f"{v} round {r}: rc {p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[0][3:])
            d.pop("kernel_src", None)
            res[v].append(d)
            if os.environ.get("AB_SHOW_PLACEMENT"):  # the kept pair's write rates, GB/s
                for k, x in d.items():
                    g, ch = x["placement"]["candidate_write_gbs"], x["placement"]["chosen"]
                    print(f"  placement {k}: kept {[g[i] for i in ch] if g else []}, best {max(g) if g else None}", flush=True)
            print(f"round {r} {v:16s} " + "  ".join(f"{k} {x['us_step']:.2f}/{x['k_step_us']:.2f}" for k, x in d.items()),
                  flush=True)
    print("median us/step (wall) per case:")
    for v in variants:
        cs = res[v][0].keys()
        med = {k: sorted(x[k]["us_step"] for x in res[v])[len(res[v]) // 2] for k in cs}
        print(f"  {v:16s} " + "  ".join(f"{k} {m:.2f}" for k, m in med.items()), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()
