"""Serial CPU baseline for bench.py (TEST INFRASTRUCTURE: the oracle timed, never the product).

Runs the oracle (a C port of the reference algorithm) on ONE core -- it is started by
bench.py as a child process with OMP_NUM_THREADS=1 so no OpenMP pool is shared with the
GPU process -- on a bounded sample of the benchmark workload and prints one JSON object.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import orc  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    geo = orc.geo_ldc(n, n, n)
    o = orc.Oracle(orc.LDC, geo, 0.55)
    o.step(1)  # warm caches / page in
    t = time.perf_counter()
    o.step(steps)
    dt = time.perf_counter() - t
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    print(json.dumps({"mlups": n ** 3 * steps / dt / 1e6, "seconds": dt, "n": n, "steps": steps,
                      "threads": int(os.environ.get("OMP_NUM_THREADS", "0") or 0), "cpu": model}))


if __name__ == "__main__":
    main()
