"""One-line summary of a bench.py JSON line: workload, ms/step, kernel ms, roofline fraction."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    r = d["roofline"]
    print(d["config"]["workload"][:40], "ms/step %.3f kernel_ms %.3f frac %.3f" % (d["ms_per_step"], r["kernel_ms"], r["frac"] or 0))
