"""One rank of tests/test_gpu_distributed.py (launched by torch.distributed.run, 2 ranks sharing cuda:0 over gloo):
the multi-GPU combine end to end through libpinot_hip -- ph_query_execute_dense into this rank's dense partial
tables, pinot_amd.distributed.reduce_tables across the ranks, ph_dense_finalize of this rank's key shard --
gathered on rank 0 and compared with the oracle over ALL segments (the GroupByCombineOperator result).

Rank r pins segments i = r (mod world) of one deterministic table.  Queries: the config-3 shape (2-column group-by
over a ~160 000-key space: COUNT / integer SUM / MIN / MAX, key-range shards on both ranks), a DOUBLE SUM group-by
(within 1e-9 relative), and config 5's DISTINCTCOUNTHLL over an inverted-index filter (aggregation only: the HLL
register max all-reduce).  Writes "OK <queries>" or the first mismatch to argv[1] on rank 0."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

QUERIES = [
    "SET numGroupsLimit=1000000; SELECT g1, g2, SUM(m), COUNT(*), MIN(m), MAX(m) FROM t WHERE f BETWEEN 0 AND 499 "
    "GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 1000000",
    "SELECT g1, SUM(d), COUNT(*), MIN(d) FROM t WHERE f < 700 GROUP BY g1 ORDER BY g1 LIMIT 1000",
    "SELECT DISTINCTCOUNTHLL(u), COUNT(*) FROM t WHERE c IN (3, 103, 203, 303)",
]
NSEG = 5


def table(i):
    rng = np.random.default_rng([0xD157, i])
    n = 120_000 + 1_111 * i
    g1 = rng.integers(0, 400, n).astype(np.int32)
    g2 = rng.integers(0, 400, n).astype(np.int32)
    g1[:400] = np.arange(400)  # complete dictionaries: identical table-level ids on every rank
    g2[:400] = np.arange(400)
    c = rng.integers(0, 1000, n).astype(np.int32)
    c[:1000] = np.arange(1000)
    return {"g1": (g1, "INT"), "g2": (g2, "INT"), "f": (rng.integers(0, 1000, n).astype(np.int32), "INT"),
            "m": (rng.integers(-5000, 1 << 20, n).astype(np.int32), "INT"),
            "d": (np.round(rng.normal(0, 100, n), 2), "DOUBLE"),
            "c": (c, "INT"), "u": (rng.integers(0, 1 << 24, n).astype(np.int32), "INT")}


def rows_match(got, exp, rtol=1e-9):
    if len(got) != len(exp):
        return f"{len(got)} rows vs {len(exp)}"
    for g, e in zip(got, exp):
        for a, b in zip(g, e):
            if a == b:
                continue
            if isinstance(b, float) and isinstance(a, float) and abs(a - b) <= rtol * max(abs(b), 1e-300):
                continue
            return f"row {g} vs {e}"
    return None


def main():
    import torch
    import torch.distributed as dist

    from oracle import oracle as O
    from pinot_amd.distributed import DistributedQuery, gather_to_root
    from pinot_amd.engine import GpuContext
    from pinot_amd.query import parse_sql
    from pinot_amd.reduce import reduce_groups
    from pinot_amd.segment import create_segment
    out_path = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    ctx = GpuContext(0)
    tables = [table(i) for i in range(NSEG)]
    mine = [ctx.pin(create_segment(f"d{i}", tables[i], inverted=("c",))) for i in range(NSEG) if i % world == rank]
    for g in ("g1", "g2"):
        ctx.set_table_dictionary(g, "INT", np.arange(400, dtype=np.int32))
    ctx.set_schema({c: t for c, (_, t) in tables[0].items()})
    runner = DistributedQuery(ctx)
    msg = None
    for sql in QUERIES:
        q = parse_sql(sql)
        res, (g0, g1), scan = runner.execute(q, mine)
        got = gather_to_root(res)
        if rank == 0 and msg is None:
            e = O.execute(q, [O.build_segment(f"d{i}", t, inverted=("c",)) for i, t in enumerate(tables)])
            rows = reduce_groups(q, got[0], got[1]).rows
            bad = rows_match(rows, reduce_groups(q, e.keys, e.aggs).rows)
            for k, a in enumerate(q.aggregations):  # HLL registers: raw, bit-exact
                if a.function == "DISTINCTCOUNTHLL" and not bad:
                    if not all(np.array_equal(x[k], y[k]) for x, y in zip(got[1], e.aggs)):
                        bad = "HLL registers differ"
            if bad:
                msg = f"{sql}: {bad}"
        if q.group_by and len(q.group_by) == 2:
            assert g1 > g0, "both ranks own a key shard of the 160 000-key space"
    dist.barrier()
    if rank == 0:
        with open(out_path, "w") as f:
            f.write(msg or f"OK {len(QUERIES)}")
    ctx.set_stream(0)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
