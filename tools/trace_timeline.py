"""Kernel timeline of a rocprofv3 --kernel-trace CSV (tuning aid): python3 tools/trace_timeline.py <kernel_trace.csv>
[first_kernel_regex] [occurrence] [count] -- prints `count` dispatches from the given occurrence of a kernel, with each
one's start offset, duration and the idle gap before it (all in microseconds)."""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    occ = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    cnt = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    hits = [i for i, e in enumerate(ev) if pat.search(e[2])]
    i0 = hits[min(occ, len(hits) - 1)]
    t0, prev_end = ev[i0][0], ev[i0][0]
    for s, e, n in ev[i0:i0 + cnt]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {(s - prev_end) / 1e3:8.1f}  {n[:90]}")
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
