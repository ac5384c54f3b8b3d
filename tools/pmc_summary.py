"""Summarise rocprofv3 --pmc passes: python tools/pmc_summary.py DIR [kernel-substring]

Averages every counter per kernel (over dispatches) across all counter_collection.csv files under DIR and
derives the ratios used in DESIGN.md: VALU / MFMA instruction mix, MFMA-busy and SQ-busy fractions, LDS
bank-conflict rate.
"""
import collections
import csv
import os
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for dp, _, fs in os.walk(root):
    for f in fs:
        if not f.endswith("counter_collection.csv"):
            continue
        for r in csv.DictReader(open(os.path.join(dp, f))):
            k = r["Kernel_Name"]
            if pat and pat not in k:
                continue
            short = k.replace("(anonymous namespace)::", "").replace("void ", "")
            short = short.split("(")[0]
            acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    c = {n: sum(v) / len(v) for n, v in acc[k].items()}
    print(k, "dispatches", max(len(v) for v in acc[k].values()))
    for n in sorted(c):
        print(f"   {n:28s} {c[n]:.6g}")
    if "SQ_INSTS_VALU" in c and "SQ_INSTS_MFMA" in c:
        print(f"   VALU/MFMA instructions       {c['SQ_INSTS_VALU'] / max(c['SQ_INSTS_MFMA'], 1):.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
        # MFMA busy cycles are summed over the 1024 SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs
        # (MI355X_MICROARCH.md: kernel cycles = GRBM_GUI_ACTIVE / 8)
        print(f"   MFMA busy fraction           {c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(c['GRBM_GUI_ACTIVE'] / 8 * 1024, 1):.3f}")
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_ACTIVE_INST_LDS" in c:
        print(f"   LDS conflict / LDS active    {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_ACTIVE_INST_LDS'], 1):.3f}")
