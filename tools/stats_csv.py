"""Print a rocprofv3 kernel_stats.csv as per-step milliseconds: python tools/stats_csv.py FILE STEPS [TOP]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:top]:
    t = float(r["TotalDurationNs"])
    print(f"{t / steps / 1e6:7.3f} ms/step {float(r['Calls']) / steps:6.1f}/step {float(r['AverageNs']) / 1e3:8.1f} us  "
          f"{r['Name'][:100]}")
print(f"total {tot / steps / 1e6:.2f} ms/step over {steps:.0f} steps")
