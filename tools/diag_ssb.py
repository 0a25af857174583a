"""GPU diagnostic: the 13 SSB queries on one bench-size lineorder segment (config4's first segment) against the
oracle, query by query, with and without PH_LIMIT_EAGER (the numGroupsLimit pass-first order).  Prints the
queries whose rows differ and the first differing rows.
    python3 tools/diag_ssb.py [rows]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench as B
    from oracle import oracle as O
    from pinot_amd.engine import GpuContext
    from pinot_amd.query import parse_sql
    from pinot_amd.reduce import reduce_groups
    from tests import workloads as W
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    t0 = time.time()
    buf = W.ssb_segment_buffers("ssb_0", rows, seed=0xC004)
    osegs = B.oracle_segments([buf])
    print(f"built {rows} rows in {time.time() - t0:.1f}s", flush=True)
    ctx = GpuContext(0)
    seg = ctx.pin(buf)
    bad = 0
    for name, sql in W.SSB_QUERIES.items():
        q = parse_sql(sql)
        res = O.execute(q, osegs, 8)
        e = reduce_groups(q, res.keys, res.aggs).rows
        for eager in (False, True):
            if eager:
                os.environ["PH_LIMIT_EAGER"] = "1"
            r = ctx.execute(q, [seg])
            os.environ.pop("PH_LIMIT_EAGER", None)
            got = reduce_groups(q, r.keys, r.aggs).rows
            ok = got == e
            print(f"{name} eager={eager} ok={ok} rows {len(got)} vs {len(e)} mode={r.stats.mode} "
                  f"kernel={r.stats.scan_kernel} limit_pass={getattr(r.stats, 'limit_pass', None)} "
                  f"reached={r.stats.num_groups_limit_reached}", flush=True)
            if not ok:
                bad += 1
                diffs = [(i, a, b) for i, (a, b) in enumerate(zip(got, e)) if a != b][:3]
                print("   first diffs:", diffs, flush=True)
    print("bad", bad, flush=True)


if __name__ == "__main__":
    main()
