"""Serial CPU baseline for bench.py (TEST INFRASTRUCTURE: the oracle timed, never the product).

Runs the oracle (oracle/lbm_oracle.c, a serial C port of the reference algorithm) pinned to ONE
host core (os.sched_setaffinity, the `taskset -c` of BASELINE.md section 4; OMP_NUM_THREADS=1 so
no OpenMP pool runs) on bounded samples and prints one JSON object:

  * `bench`: LDC n^3 (the bench workload, 512^3 by default), `steps` steps after the set-up;
  * `c1`:    LDC 64^3, config C1, 200 fixed steps;
  * `c1_converge` (with --converge): C1 to convergence (tol 1e-6, 50 hits, max 10000).

    python oracle/cpu_baseline.py [n] [steps] [--converge]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pin_one_core() -> int:
    """Pin this process to the highest-numbered core it may run on (away from core 0, where
    the GPU process's host threads tend to sit); returns that core."""
    cores = sorted(os.sched_getaffinity(0))
    core = cores[-1]
    os.sched_setaffinity(0, {core})
    return core


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def timed_ldc(n: int, steps: int):
    import orc
    o = orc.Oracle(orc.LDC, orc.geo_ldc(n, n, n), 0.55)
    t = time.perf_counter()
    o.step(steps)
    dt = time.perf_counter() - t
    return {"mlups": n ** 3 * steps / dt / 1e6, "seconds": round(dt, 3), "n": n, "steps": steps}


def converge_ldc(n: int = 64):
    import orc
    o = orc.Oracle(orc.LDC, orc.geo_ldc(n, n, n), 0.55)
    t = time.perf_counter()
    k, res = o.run_converge(10000, 50, 1e-6)
    dt = time.perf_counter() - t
    return {"mlups": n ** 3 * k / dt / 1e6, "seconds": round(dt, 3), "n": n, "steps": int(k), "residual": res}


def main():
    os.environ["OMP_NUM_THREADS"] = "1"
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 512
    steps = int(args[1]) if len(args) > 1 else 1
    core = pin_one_core()
    out = {"core": core, "threads": 1, "cpu": cpu_model()}
    out["c1"] = timed_ldc(64, 200)
    out["bench"] = timed_ldc(n, steps)
    if "--converge" in sys.argv:
        out["c1_converge"] = converge_ldc(64)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
