"""Per-kernel sums of the SQ counters collected by tools/gpu_sq.sh.   python3 tools/sq_summary.py <dir>"""
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")[:60]
        if "k_scan" not in k and "k_part" not in k:
            continue
        acc.setdefault(k, {})
        c = row["Counter_Name"]
        acc[k][c] = acc[k].get(c, 0.0) + float(row.get("Counter_Value", 0) or 0)
for k, v in acc.items():
    print(k)
    for c in sorted(v):
        print(f"   {c:28s} {v[c]:.4g}")
