"""Per-kernel sums of the SQ counters collected by tools/gpu_sq.sh.   python3 tools/sq_summary.py <dir>"""
import csv
import glob
import os
import sys

d = sys.argv[1]
acc, disp = {}, {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")[:60]
        if "ph::k_" not in k:
            continue
        acc.setdefault(k, {})
        c = row["Counter_Name"]
        acc[k][c] = acc[k].get(c, 0.0) + float(row.get("Counter_Value", 0) or 0)
        disp.setdefault((k, c), set()).add(row.get("Dispatch_Id", ""))
for k, v in acc.items():
    print(k)
    for c in sorted(v):
        n = max(1, len(disp.get((k, c), ())))
        print(f"   {c:28s} {v[c]:.4g}   per dispatch {v[c] / n:.4g}  ({n} dispatches)")
