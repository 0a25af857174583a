"""Where a query's wall time goes on the host: the C++ call vs the Python mirror around it (tuning aid).
    python3 tools/py_overhead.py config3-agg"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import bench as B
    from pinot_amd.engine import GpuContext
    from pinot_amd.query import parse_sql
    w = sys.argv[1] if len(sys.argv) > 1 else "config3-agg"
    if os.environ.get("WITH_TORCH"):  # the bench's process: torch (and its bundled HIP runtime) initialised first
        import torch
        torch.cuda.init()
        torch.zeros(1, device="cuda")
    query, cols, _ = B.WORKLOADS[w]
    q = parse_sql(query)
    ctx = GpuContext(0)
    pinned = [ctx.pin(B.make_segment_buffers(i, 10_000_000, seed=1000, cols=cols)) for i in range(100)]
    for _ in range(3):
        ctx.execute(q, pinned, copy=False)
    n = 50
    t = time.perf_counter()
    host = []
    for _ in range(n):
        r = ctx.execute(q, pinned, copy=False)
        host.append(r.stats.host_ms + r.stats.device_ms)
    wall = (time.perf_counter() - t) * 1e3 / n
    print(f"{w}: wall {wall:.3f} ms per query, C++ call (host_ms + device_ms) {np.mean(host):.3f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        r = ctx.execute(q, pinned, copy=False)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(12)


if __name__ == "__main__":
    main()
