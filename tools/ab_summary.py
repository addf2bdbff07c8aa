#!/usr/bin/env python3
"""Summarise tools/ab_profile.sh output: per variant the bench value, k_step's median launch
time (kernel trace) and median HBM read bytes per launch (FETCH_SIZE x 2, gfx950 correction).
    python3 tools/ab_summary.py gpurun_out/ab_<tag> [variant ...]"""
import csv
import glob
import json
import os
import statistics as st
import sys

root = sys.argv[1]
names = sys.argv[2:] or sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
for v in names:
    d = os.path.join(root, v)
    j = [json.loads(line) for line in open(d + ".json") if line.startswith("{")]
    fe = [float(r["Counter_Value"]) for r in csv.DictReader(open(glob.glob(d + "/fetch/*counter_collection.csv")[0]))
          if "k_step" in r["Kernel_Name"]]
    kt = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
          for r in csv.DictReader(open(glob.glob(d + "/kt/*kernel_trace.csv")[0])) if "k_step" in r["Kernel_Name"]]
    print(f"{v:10s} bench {j[0]['value'] if j else None} MLUPS  k_step median {st.median(kt):.4f} ms ({len(kt)})  "
          f"read {st.median(fe) * 1024 * 2 / 1e9:.3f} GB/launch ({len(fe)})")
