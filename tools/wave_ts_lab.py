#!/usr/bin/env python3
"""Where a launch's time goes: per-wave start / end timestamps of the 4-cell chunk waves
(tools/lab_build.py wave_ts: s_memrealtime, 100 MHz) over one step, summarised as wave lifetimes,
occupancy over time and the completion rate (measurement tool; LBM_LIBRARY = the wave_ts build).

    LBM_LIBRARY=tools/ab/wave_ts/liblbm.so python3 tools/wave_ts_lab.py c3 ldc256 ldc512
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
import torch  # noqa: F401,E402
import lbm_amd  # noqa: E402
from lbm_amd import cases  # noqa: E402

for kv in filter(None, os.environ.get("AB_TUNE", "").split(",")):
    k, v = kv.split(":")
    lbm_amd.tune(int(k), int(v))


def make(w):
    if w == "c3":
        return cases.poiseuille(128, 512, 128)[0]
    n = int(w[3:])
    return cases.ldc_device(n, n, n)


def summarise(w):
    lat = make(w)
    n = lat.layout()["active_chunks"]
    lat.step(20, history=False)
    lat.sync()
    lat.step(1, history=False)
    lat.sync()
    n = min(n, 1 << 20)
    buf = (C.c_ulonglong * (2 * n))()
    rc = lbm_amd.lbm_lib().lbm_lab_ts_copy(buf, 2 * n)
    assert rc == 0, rc
    lat.close()
    ts = np.frombuffer(buf, dtype=np.uint64).reshape(n, 2).copy()
    grp = (ts[:, 1] >> np.uint64(56)).astype(np.int64)  # the block's XCD group (dispatch index mod 8)
    xcc = (ts[:, 0] >> np.uint64(56)).astype(np.int64)  # HW_REG_XCC_ID of the wave's XCD
    ts[:, 0] &= np.uint64((1 << 56) - 1)
    ts[:, 1] &= np.uint64((1 << 56) - 1)
    ts = ts.astype(np.int64)
    t0 = ts[:, 0].min()
    s = (ts[:, 0] - t0) / 100.0  # us (100 MHz)
    e = (ts[:, 1] - t0) / 100.0
    life = e - s
    span = e.max()
    order = np.sort(e)
    mid = order[int(0.25 * n)], order[int(0.75 * n)]
    rate = 0.5 * n / (mid[1] - mid[0])  # waves per us in the middle half
    bins = np.arange(0.0, span + 2.0, 2.0)
    occ = [int(((s <= b) & (e > b)).sum()) for b in bins]
    return {"lattice": w, "waves": n, "span_us": round(span, 2),
            "lifetime_us": {"mean": round(life.mean(), 2), "p10": round(np.percentile(life, 10), 2),
                            "p50": round(np.percentile(life, 50), 2), "p90": round(np.percentile(life, 90), 2)},
            "first_end_us": round(order[0], 2), "last_start_us": round(s.max(), 2),
            "mid_rate_waves_per_us": round(rate, 1), "ideal_us_at_mid_rate": round(n / rate, 2),
            "lifetime_by_decile_of_start_us": [round(float(life[(s >= np.percentile(s, 10 * k)) &
                                                              (s <= np.percentile(s, 10 * k + 10))].mean()), 2)
                                               for k in range(10)],
            "occupancy_every_2us": occ,
            "by_xcd_group": [{"waves": int((grp == g).sum()), "first_start_us": round(float(s[grp == g].min()), 2),
                              "last_start_us": round(float(s[grp == g].max()), 2),
                              "last_end_us": round(float(e[grp == g].max()), 2),
                              "p99_end_us": round(float(np.percentile(e[grp == g], 99)), 2),
                              "mean_life_us": round(float(life[grp == g].mean()), 2),
                              "xcc": sorted(set(int(v) for v in xcc[grp == g]))}
                             for g in range(8) if (grp == g).any()]}


for w in sys.argv[1:]:
    print(json.dumps(summarise(w)), flush=True)
