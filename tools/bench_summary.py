#!/usr/bin/env python3
"""Print the headline and secondary lines of a bench.py JSON output (the last line starting
with '{'):  python3 tools/bench_summary.py gpurun_out/<tag>/bench.json"""
import json
import sys

p = None
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        p = json.loads(ln)
r = p["roofline"]
print(f"headline {p['value']} MLUPS, {p['ms_per_step']} ms/step, frac {r['frac']} (k_step {r['avg_kernel_ms']} ms), "
      f"traffic {r['traffic']}, probe {r['stream_probe_gbs']} ({r['frac_of_stream_probe']}), setup {p['setup']}")
for k, v in p.get("secondary", {}).items():
    rl = v.get("roofline", {})
    ro = rl.get("rocprof", {})
    m = v.get("mlups_nlattice") or v.get("mlups_box") or v.get("mlups")
    print(f"  {k:48s} {m:>10} MLUPS  wall {v.get('ms_per_step')} ms  step {rl.get('step_us')} us  frac {rl.get('frac')}"
          f"  rocprof {ro.get('k_step_us')}/{ro.get('k_nee_fix_us')} frac {ro.get('frac_k_step')}  nee {v.get('nee_values')}")
    if "fresh_lattices" in v:
        print("     fresh lattices", v["fresh_lattices"]["step_us_min_median_max"], v["fresh_lattices"]["frac_min_median_max"],
              [x["kept_write_gbs"] for x in v["fresh_lattices"]["per_lattice"]])
cb = p.get("cpu_baseline")
if cb:
    print("cpu", cb["value"], {k: cb[k]["mlups"] for k in ("c1", "c1_converge", "c2", "c3") if k in cb})
