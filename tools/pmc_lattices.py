#!/usr/bin/env python3
"""Summarise tools/pmc_lattices.sh: per lattice, k_step's mean launch time, HBM bytes per launch
(FETCH_SIZE x 2, the gfx950 correction for 16-B streaming reads, + WRITE_SIZE; KiB -> B) against
the algorithmic 152 B x fluid cells, and its SQ counters per launch.

    python3 tools/pmc_lattices.py gpurun_out/pmcl_<tag> <tag> [--merge]

Writes profiles/<tag>_lattices.json; --merge also records each lattice in profiles/pmc_traffic.json
(read by bench.py for the secondary lines' traffic ratios)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {"c3": "poiseuille_128x512x128 (C3)", "c4": "bifurcation_64x83x32 (C4)",
         "c4x4": "bifurcation_x4_256x332x128 (C4 upsampled)", "coronary": "coronary_291x291x372 (synthetic vessel)",
         "ldc64": "ldc_64^3", "ldc256": "ldc_256^3 (C2)", "ldc512": "ldc_512^3",
         "c5": "ldc_512x512x4096 (C5 lattice)"}


def counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(path):
        for r in csv.DictReader(open(f)):
            if "k_step" in r["Kernel_Name"]:
                acc[r["Counter_Name"]][r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    # per dispatch: sum over the counter's instances (XCDs / SEs), then the mean over dispatches
    return {k: sum(sum(v) for v in d.values()) / len(d) for k, d in acc.items() if d}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out = {}
    for case in sorted(os.listdir(src)):
        d = os.path.join(src, case)
        if not os.path.isdir(d):
            continue
        abl = [json.loads(ln[3:]) for ln in open(os.path.join(d, "kt.json")) if ln.startswith("AB ")][0]
        ab = abl[case]
        kt = [r for r in csv.DictReader(open(glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))[0]))
              if "k_step" in r["Name"]]
        calls = sum(int(r["Calls"]) for r in kt)
        avg_ns = sum(float(r["TotalDurationNs"]) for r in kt) / max(1, calls)
        fx = [r for r in csv.DictReader(open(glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))[0]))
              if "k_nee_fix" in r["Name"]]
        fix_ns = sum(float(r["TotalDurationNs"]) for r in fx) / max(1, sum(int(r["Calls"]) for r in fx))
        fe = counters(os.path.join(d, "fetch", "*counter_collection.csv")).get("FETCH_SIZE", 0.0)
        wr = counters(os.path.join(d, "write", "*counter_collection.csv")).get("WRITE_SIZE", 0.0)
        sq = counters(os.path.join(d, "sq", "*counter_collection.csv"))
        rd_b, wr_b = fe * 1024 * 2, wr * 1024
        algo = 152.0 * ab["n_fluid"]
        out[case] = {
            "lattice": NAMES.get(case, case), "n_fluid": ab["n_fluid"], "launch_shape": ab["launch_shape"],
            "k_step_avg_us": round(avg_ns / 1e3, 3), "k_step_launches": calls,
            "read_bytes": int(rd_b), "write_bytes": int(wr_b), "bytes_per_launch": int(rd_b + wr_b),
            "algo_bytes_per_launch": int(algo), "traffic_over_algo": round((rd_b + wr_b) / algo, 3) if algo else None,
            "achieved_algo_gbs": round(algo / avg_ns, 1) if avg_ns else None,
            "frac_of_8tbs": round(algo / avg_ns / 8000.0, 4) if avg_ns else None,
            "k_nee_fix_avg_us": round(fix_ns / 1e3, 3) if fx else None,
            "sq_per_launch": {k: round(v, 1) for k, v in sorted(sq.items())},
            # 1024 SIMDs; SQ_WAIT_ANY / SQ_WAVE_CYCLES: the share of wave-cycles spent waiting
            "waves_per_simd": round(sq["SQ_WAVES"] / 1024.0, 2) if sq.get("SQ_WAVES") else None,
            "wait_share": round(sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"], 3) if sq.get("SQ_WAVE_CYCLES") else None,
            "reads_over_algo": round(rd_b / (76.0 * ab["n_fluid"]), 3) if ab["n_fluid"] else None,
            "tag": tag, "kernel_src": abl.get("kernel_src"),
        }
        print(case, json.dumps(out[case]))
    with open(os.path.join(REPO, "profiles", f"{tag}_lattices.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    if "--merge" in sys.argv:
        p = os.path.join(REPO, "profiles", "pmc_traffic.json")
        cur = json.load(open(p))
        for case, v in out.items():
            cur[NAMES.get(case, case)] = v
        with open(p, "w") as f:
            json.dump(cur, f, indent=1)


if __name__ == "__main__":
    main()
