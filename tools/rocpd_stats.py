#!/usr/bin/env python3
"""Per-kernel launch statistics from rocprofv3's SQLite output (run_results.db), the figures
its --stats CSV gives: calls, mean / min / max duration (us), share of kernel time.

    python3 tools/rocpd_stats.py <dir or .db> [top]
"""
import glob
import os
import sqlite3
import sys


def stats(path, top=8):
    db = path if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    con = sqlite3.connect(db)
    rows = list(con.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                            "max(end - start) from kernels group by name order by sum(end - start) desc"))
    total = sum(r[2] for r in rows) or 1
    return [{"kernel": r[0], "calls": r[1], "avg_us": round(r[3] / 1e3, 3), "min_us": round(r[4] / 1e3, 3),
             "max_us": round(r[5] / 1e3, 3), "pct": round(100.0 * r[2] / total, 2)} for r in rows[:top]]


if __name__ == "__main__":
    for r in stats(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8):
        print(f"{r['calls']:6d} {r['avg_us']:10.3f} {r['min_us']:10.3f} {r['max_us']:10.3f} {r['pct']:6.2f}%  {r['kernel'][:110]}")
