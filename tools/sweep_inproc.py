"""Tuning-knob sweep in ONE process: pins a bench.py workload once, then runs the query under each environment
setting (the library reads its PH_* knobs with getenv at every query) and prints device ms per setting.
    python3 tools/sweep_inproc.py config3 "-" "PH_PART_BATCH_ROWS=500000000" "PH_TILE_WORDS=16,PH_PART_KLO=13"
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench as B
    from pinot_amd.engine import GpuContext
    from pinot_amd.query import parse_sql
    w = sys.argv[1]
    settings = sys.argv[2:] or ["-"]
    query, cols, _ = B.WORKLOADS[w]
    rows = int(os.environ.get("SWEEP_ROWS", "1000000000"))
    nseg = rows // 10_000_000
    q = parse_sql(query)
    ctx = GpuContext(0)
    t0 = time.time()
    pinned = [ctx.pin(B.make_segment_buffers(i, 10_000_000, seed=1000, cols=cols)) for i in range(nseg)]
    for g in q.group_by:
        ctx.set_table_dictionary(g, "INT", np.arange(cols[g][0], dtype=np.int32))
    print(f"pinned {nseg} segments in {time.time() - t0:.1f}s", flush=True)
    ref = None
    for s in settings:
        keys = [kv.split("=", 1)[0] for kv in s.split(",")] if s != "-" else []
        for kv in (s.split(",") if s != "-" else []):
            k, v = kv.split("=", 1)
            os.environ[k] = v
        iters = int(os.environ.get("SWEEP_ITERS", "8"))
        for _ in range(2 if iters > 1 else 0):
            r = ctx.execute(q, pinned, copy=False)
        ms = []
        for _ in range(iters):
            r = ctx.execute(q, pinned, copy=False)
            ms.append(r.stats.device_ms)
        sig = (r.num_groups, float(np.sum(r.agg_columns[0])) if r.agg_columns else 0.0)
        ok = ref is None or sig == ref
        ref = ref or sig
        print(f"{s:60s} device_ms median {np.median(ms):.3f} min {np.min(ms):.3f} mode {r.stats.mode} kernel {r.stats.scan_kernel} "
              f"{'same result' if ok else 'RESULT DIFFERS'}", flush=True)
        for k in keys:
            del os.environ[k]


if __name__ == "__main__":
    main()
