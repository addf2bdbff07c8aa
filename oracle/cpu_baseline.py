"""Serial CPU baseline for bench.py (TEST INFRASTRUCTURE: the oracle timed, never the product).

Runs the oracle (oracle/lbm_oracle.c, a serial C port of the reference algorithm) on bounded
samples, each in its own process pinned to ONE host core (os.sched_setaffinity, the `taskset -c`
of BASELINE.md section 4; OMP_NUM_THREADS=1 so no OpenMP pool runs).  The samples run side by
side on distinct cores (the highest-numbered ones this process may use, away from the GPU
process's host threads), so their wall time is the longest one's; each is still one serial
core's throughput.  Prints one JSON object:

  * `bench`:        LDC n^3 (the bench workload, 512^3 by default), `steps` steps after set-up;
  * `c1`:           LDC 64^3, config C1, 200 fixed steps;
  * `c1_converge`:  C1 to convergence (tol 1e-6, 50 hits, max 10000) with the residual summed in
                    fp64, liblbm's default order, so it stops at liblbm's step (5080);
  * `c2`:           LDC 256^3 (config C2), 10 fixed steps (C2 scaled down
                    from 1000 steps, which would take ~25 min on one core);
  * `c3`:           Poiseuille 128 x 512 x 128 (config C3), 20 fixed steps (scaled down likewise).

    python oracle/cpu_baseline.py [n] [steps] [--quick]      # --quick: bench + c1 only
    python oracle/cpu_baseline.py --sample NAME CORE [n steps]  # one sample (internal)
"""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

SAMPLES = ("c1_converge", "c2", "bench", "c3", "c1")  # longest first: they start together


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def timed(o, cells: int, steps: int, **extra):
    t = time.perf_counter()
    o.step(steps)
    dt = time.perf_counter() - t
    return {"mlups": cells * steps / dt / 1e6, "seconds": round(dt, 3), "steps": steps, **extra}


def run_sample(name: str, n: int = 512, steps: int = 1):
    import orc
    if name in ("bench", "c1", "c2"):
        m = {"bench": n, "c1": 64, "c2": 256}[name]
        k = {"bench": steps, "c1": 200, "c2": 10}[name]
        return timed(orc.Oracle(orc.LDC, orc.geo_ldc(m, m, m), 0.55), m ** 3, k, n=m)
    if name == "c3":
        geo = orc.geo_poiseuille(128, 512, 128)
        nlat, _ = orc.index_transform(geo)
        out = timed(orc.Oracle(orc.POISEUILLE, geo, 0.58), geo.size, 20, shape_xyz=[128, 512, 128])
        out["mlups_nlattice"] = out["mlups"] * nlat / geo.size
        return out
    if name == "c1_converge":
        o = orc.Oracle(orc.LDC, orc.geo_ldc(64, 64, 64), 0.55)
        o.residual_fp64(True)
        t = time.perf_counter()
        k, res = o.run_converge(10000, 50, 1e-6)
        dt = time.perf_counter() - t
        return {"mlups": 64 ** 3 * k / dt / 1e6, "seconds": round(dt, 3), "n": 64, "steps": int(k), "residual": res}
    raise SystemExit(f"unknown sample {name}")


def main():
    os.environ["OMP_NUM_THREADS"] = "1"
    if sys.argv[1:2] == ["--sample"]:
        name, core = sys.argv[2], int(sys.argv[3])
        os.sched_setaffinity(0, {core})
        rest = [int(a) for a in sys.argv[4:]]
        print(json.dumps(run_sample(name, *rest)))
        return
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 512
    steps = int(args[1]) if len(args) > 1 else 1
    names = ("bench", "c1") if "--quick" in sys.argv else SAMPLES
    cores = sorted(os.sched_getaffinity(0))[::-1]
    kids = {}
    for i, name in enumerate(names):
        core = cores[i % len(cores)]
        cmd = [sys.executable, __file__, "--sample", name, str(core)] + ([str(n), str(steps)] if name == "bench" else [])
        kids[name] = (core, subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True))
    out = {"threads_per_sample": 1, "cpu": cpu_model(), "cores": {}}
    for name, (core, p) in kids.items():
        so, _ = p.communicate()
        if p.returncode != 0:
            raise SystemExit(f"cpu baseline sample {name} failed ({p.returncode})")
        out[name] = json.loads(so.strip().splitlines()[-1])
        out["cores"][name] = core
    out["core"] = out["cores"]["bench"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
