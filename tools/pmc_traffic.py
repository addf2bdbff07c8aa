#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run into profiles/.

    python tools/pmc_traffic.py gpurun_out/prof_<tag> <tag>

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.csv            per-kernel FETCH_SIZE / WRITE_SIZE averages
  profiles/pmc_traffic.json         HBM bytes per launch of the dominant kernel, read by bench.py

HBM bytes follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE and WRITE_SIZE are in KiB
(from the L2's memory-side request counters, each collected in its own --pmc pass);
on gfx950 FETCH_SIZE counts exactly half of a wide (16 B/lane) streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAIN = "k_step"
FIX = "k_reduce_slices"


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def find(d, sub):
    for k, v in d.items():
        if sub in k:
            return k, v
    return None, (None, 0)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(src, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "FETCH_SIZE_KiB_avg", "WRITE_SIZE_KiB_avg",
                    "hbm_read_bytes_corrected", "hbm_write_bytes"])
        for k in sorted(set(fetch) | set(write)):
            fk, n = fetch.get(k, (0.0, 0))
            wk, _ = write.get(k, (0.0, 0))
            w.writerow([k, n, f"{fk:.1f}", f"{wk:.1f}", int(fk * 1024 * 2), int(wk * 1024)])
    durations = {}
    with open(stats) as f:
        for r in csv.DictReader(f):
            durations[r["Name"]] = float(r["AverageNs"])
    out = {}
    for name in (MAIN, FIX):
        k, (fk, n) = find(fetch, name)
        _, (wk, _) = find(write, name)
        if k is None:
            continue
        _, dur = find(durations, name)
        rd, wr = fk * 1024 * 2, wk * 1024
        out[name] = {"kernel": k, "dispatches": n, "read_bytes": int(rd), "write_bytes": int(wr),
                     "bytes_per_launch": int(rd + wr), "avg_duration_ns": dur}
    wl = os.environ.get("LBM_WORKLOAD", "ldc_512x512x512_per_gpu")
    ksrc = None  # the bench line of the kernel-trace pass names the kernels it ran
    for ln in open(os.path.join(src, "kt.log")):
        if ln.startswith("{") and '"kernel_src"' in ln:
            ksrc = json.loads(ln)["kernel_src"]
    path = os.path.join(prof, "pmc_traffic.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[wl] = dict(out.get(MAIN, {}), tag=tag, kernel_src=ksrc, reduce=out.get(FIX),
                 note="FETCH_SIZE x2 (gfx950 half-count of 16-B/lane streaming reads) + WRITE_SIZE, KiB->B; "
                      "separate --pmc passes of bench.py --steps 20 --warmup 5")
    json.dump(d, open(path, "w"), indent=1)
    print(json.dumps(d[wl], indent=1))


if __name__ == "__main__":
    main()
