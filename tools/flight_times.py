"""Per-query device time / plan mode of the config4 SSB flight (tuning aid):
    python3 tools/flight_times.py [segments] [distinct]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    from pinot_amd.engine import GpuContext
    from pinot_amd.query import parse_sql
    from tests import workloads as W
    nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    distinct = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    inv = () if os.environ.get("FLIGHT_NO_INVERTED") else W.SSB_INVERTED
    built = [W.ssb_segment_buffers(f"ssb_{j}", 10_000_000, seed=0xC004 + j, inverted=inv) for j in range(distinct)]
    ctx = GpuContext(0)
    pinned = [ctx.pin(built[i % distinct]) for i in range(nseg)]
    only = os.environ.get("FLIGHT_ONLY")
    queries = dict(W.SSB_QUERIES)
    if os.environ.get("FLIGHT_SQL"):  # ad-hoc variants: "sql;;sql;;..."
        queries = {f"X{i}": q for i, q in enumerate(os.environ["FLIGHT_SQL"].split(";;"))}
    for name, sql in queries.items():
        if only and name not in only.split(","):
            continue
        q = parse_sql(sql)
        for _ in range(2):
            ctx.execute(q, pinned, copy=False)
        ms, wall = [], []
        for _ in range(3):
            t = time.perf_counter()
            r = ctx.execute(q, pinned, copy=False)
            wall.append((time.perf_counter() - t) * 1e3)
            ms.append(r.stats.device_ms)
        print(f"{name} mode {r.stats.mode} groups {r.num_groups:7d} device {np.median(ms):8.3f} ms  wall "
              f"{np.median(wall):8.3f} ms", flush=True)


if __name__ == "__main__":
    main()
