"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite) into a per-kernel stats CSV.

usage: python tools/prof_summary.py RUN_results.db OUT.csv [--steps N]
Columns follow rocprofv3's kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs, StdDev); with --steps the per-step milliseconds are printed too.
"""
import argparse
import csv
import math
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("out")
ap.add_argument("--steps", type=int, default=0, help="number of bench steps in the trace (warmup + timed)")
args = ap.parse_args()
c = sqlite3.connect(args.db)
rows = {}
for name, dur in c.execute("select name, duration from kernels"):
    rows.setdefault(name, []).append(dur)
total = sum(sum(v) for v in rows.values())
stats = []
for name, v in rows.items():
    n = len(v)
    s = sum(v)
    mean = s / n
    sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
    stats.append((name, n, s, mean, 100.0 * s / total, min(v), max(v), sd))
stats.sort(key=lambda r: -r[2])
with open(args.out, "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for r in stats:
        w.writerow([r[0], r[1], r[2], round(r[3], 3), round(r[4], 3), r[5], r[6], round(r[7], 3)])
for r in stats[:40]:
    per = f"{r[2] / args.steps / 1e6:8.3f} ms/step" if args.steps else ""
    print(f"{r[4]:6.2f}%  {r[1]:6d} x {r[3] / 1e3:9.2f} us  {per}  {r[0][:110]}")
print(f"total kernel time {total / 1e6:.2f} ms" + (f" = {total / args.steps / 1e6:.2f} ms/step" if args.steps else ""))
