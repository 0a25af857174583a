"""Per-query wall / device / host split of the SSB flight (tuning aid; the library's PH_HOST_TIMES phase stamps go to
stderr).  python3 tools/ssb_host_times.py [config4|config4-scan] [segments]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    torch.zeros(1, device="cuda")
    from pinot_amd.engine import GpuContext
    from pinot_amd.query import parse_sql
    from tests import workloads as W
    w = sys.argv[1] if len(sys.argv) > 1 else "config4"
    nseg = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    inverted = () if w.endswith("-scan") else W.SSB_INVERTED
    built = [W.ssb_segment_buffers(f"ssb_{j}", 10_000_000, seed=0xC004 + j, inverted=inverted) for j in range(4)]
    ctx = GpuContext(0)
    pinned = [ctx.pin(built[i % 4]) for i in range(nseg)]
    queries = {k: parse_sql(v) for k, v in W.SSB_QUERIES.items()}
    for g in dict.fromkeys(g for q in queries.values() for g in q.group_by):
        vals = np.unique(np.concatenate([b.columns[g].dictionary_values for b in built]))
        ctx.set_table_dictionary(g, built[0].columns[g].data_type, vals)
    ctx.set_schema({c: cb.data_type for c, cb in built[0].columns.items()})
    for _ in range(3):
        for q in queries.values():
            ctx.execute(q, pinned, copy=False)
    tot = [0.0, 0.0, 0.0]
    for name, q in queries.items():
        walls = []
        for _ in range(5):
            t = time.perf_counter()
            r = ctx.execute(q, pinned, copy=False)
            walls.append((time.perf_counter() - t) * 1e3)
        wall = float(np.median(walls))
        tot[0] += wall
        tot[1] += r.stats.device_ms
        tot[2] += r.stats.host_ms
        print(f"{name:6s} wall {wall:7.3f}  device {r.stats.device_ms:7.3f}  host {r.stats.host_ms:7.3f}  "
              f"mode {r.stats.mode}", flush=True)
    print(f"flight wall {tot[0]:.3f} device {tot[1]:.3f} host {tot[2]:.3f}", flush=True)
    if os.environ.get("STAMPS"):
        os.environ["PH_HOST_TIMES"] = "1"
        for name, q in list(queries.items())[:13]:
            print(f"--- {name}", file=sys.stderr, flush=True)
            ctx.execute(q, pinned, copy=False)


if __name__ == "__main__":
    main()
