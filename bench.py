"""Benchmark of the segment filter -> group-by hot path (BASELINE.json metric "filter+group-by rows/s and achieved
HBM GB/s, 1B rows"; headline = configs[2] with SURVEY.md 8(d)'s filter, "filter+group-by SUM query"):

    SET numGroupsLimit=2000000; SET minServerGroupTrimSize=-1; SET minSegmentGroupTrimSize=-1;
    SELECT g1, g2, SUM(m), COUNT(*), MIN(m), MAX(m) FROM t WHERE f BETWEEN 0 AND 499
    GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 2000000

over 1e9 synthetic rows per GPU in 100 segments x 10M docs: g1, g2 INT uniform over 1000 values (b = 10),
m INT through a 65 536-entry dictionary over [0, 2^20) (b = 16), f INT uniform over 1000 values (b = 10).
Algorithmic bytes = sum over the 4 referenced columns of ceil(N*b/8) = 5.75 GB per GPU.

A step = one full query: plan + the batched scan kernels over every segment of this GPU + (N > 1) the RCCL
reduce-scatter of the dense partial tables by key range + finalising this rank's key shard into host result
columns (~1M groups at N = 1).  Segments are pinned in HBM before timing.  Multi-GPU: one process per GPU and
ONE 1e9-row table of 100 segments sharded across the ranks (segment i on rank i mod N: equal rows per
segment, so this is the greedy-by-rows assignment), i.e. strong scaling -- the N = 1 line is the same query
over the same data as every other N.

`roofline.kernel_ms` is the device time of the scan kernels of one step, taken with HIP events recorded on the
stream the kernels run on (ph_exec_stats.device_ms); `traffic` is read from the PMC summary under profiles/
(tools/gpu_pmc.sh) when one exists for the workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# workload -> (query, columns {name: (cardinality, bits)}, description)
WORKLOADS = {
    # headline (BASELINE.json configs[2] with the SURVEY 8(d) filter): ~1M groups
    "config3": ("SET numGroupsLimit=2000000; SET minServerGroupTrimSize=-1; SET minSegmentGroupTrimSize=-1; "
                "SELECT g1, g2, SUM(m), COUNT(*), MIN(m), MAX(m) FROM t WHERE f BETWEEN 0 AND 499 "
                "GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 2000000",
                {"g1": (1000, 10), "g2": (1000, 10), "m": (65536, 16), "f": (1000, 10)},
                "config3: WHERE f BETWEEN 0 AND 499 GROUP BY g1, g2 (1e6 groups) SUM(m), COUNT(*), MIN(m), MAX(m)"),
    # BASELINE.json configs[1]: pure unpack + predicate scan, b = 20
    "config2": ("SELECT COUNT(*) FROM t WHERE v BETWEEN 100000 AND 199999",
                {"v": (1 << 20, 20)}, "config2: COUNT(*) WHERE v BETWEEN (10% of a 2^20 domain), b = 20"),
    # SURVEY 8(d) config 3 LDS-regime variant: g1 only with C = 100
    "config3-lds": ("SELECT g1, SUM(m), COUNT(*), MIN(m), MAX(m) FROM t WHERE f BETWEEN 0 AND 499 "
                    "GROUP BY g1 ORDER BY g1 LIMIT 1000",
                    {"g1": (100, 7), "m": (65536, 16), "f": (1000, 10)},
                    "config3-lds: WHERE f BETWEEN 0 AND 499 GROUP BY g1 (C=100) SUM/COUNT/MIN/MAX(m)"),
    # aggregation-only over the config-3 metric
    "config3-agg": ("SELECT SUM(m), COUNT(*), MIN(m), MAX(m) FROM t WHERE f BETWEEN 0 AND 499",
                    {"m": (65536, 16), "f": (1000, 10)}, "config3-agg: WHERE f BETWEEN 0 AND 499 SUM/COUNT/MIN/MAX(m)"),
}
# workloads whose segments come from tests/workloads.py value generators through create_segment (sorted columns,
# inverted indexes): (query, builder(seg_index, rows) -> SegmentBuffers, distinct segments, default rows,
# default segment rows, description)
BUILT = {
    # BASELINE.json configs[0]: the README AdAnalytics query on one 10M-row segment (sorted daysSinceEpoch)
    "config1": ("ads", 1, 10_000_000, 10_000_000,
                "config1: README AdAnalytics, sorted daysSinceEpoch range + accountId IN, GROUP BY day, one segment"),
    # BASELINE.json configs[4] on one GPU: the 4B-row table (400 x 10M-row segments, ~26 GB pinned), DISTINCTCOUNTHLL(u),
    # u at b = 24, WHERE c IN (10 ids) on an inverted index (~1 % selectivity); 4 distinct 10M-row segments pinned 100
    # times each (segment build is ~6 s each)
    "config5": ("hll", 4, 4_000_000_000, 10_000_000,
                "config5: DISTINCTCOUNTHLL(u) (b=24) WHERE c IN (10 ids) via inverted bitmaps, 1 % selectivity, 4B rows"),
}
# BASELINE.json configs[3]: the 13 SSB queries as one flight over a denormalised lineorder table (SF100 = 600M rows,
# 60 x 10M-row segments: 4 distinct segments built in dictId form by tests/workloads.py, pinned 15 times each)
FLIGHTS = {"config4": (4, 600_000_000, 10_000_000,
                       "config4: SSB lineorder SF100 flight Q1.1-Q4.3 (13 queries), the 9 string dimensions with "
                       "inverted indexes (tests/workloads.py SSB_INVERTED, as the parity tests)"),
           # SURVEY 8(d)'s config 4 as specified: every column dictionary-encoded, no inverted index (scan leaves)
           "config4-scan": (4, 600_000_000, 10_000_000,
                            "config4-scan: SSB lineorder SF100 flight Q1.1-Q4.3 (13 queries), every column a "
                            "dictionary-encoded scan leaf (no inverted index, SURVEY 8(d))")}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
MODE_NAMES = {0: "MODE_COUNT", 1: "MODE_AGG", 2: "MODE_GROUP_LDS", 3: "MODE_GROUP_GLOBAL", 4: "MODE_PARTITION",
              5: "MODE_GROUP_HASH"}
CPU_NOTE = ("threads = this job's CPU share on the GPU box (OMP_NUM_THREADS; the pool gives one GPU job 16 CPUs and "
            "asks GPU jobs to size worker pools to it), not the machine's host_cores; value_t1 is the one-thread rate")


def kernel_name(mode, scan_kernel):
    """The scan kernel that ran (ph_exec_stats.scan_kernel), with its plan mode for the generic k_scan."""
    from pinot_amd.engine import SCAN_KERNEL_NAMES
    name = SCAN_KERNEL_NAMES.get(scan_kernel, "k_scan")
    if scan_kernel == 1:
        name = f"k_scan<{MODE_NAMES.get(mode, mode)}>"
    if scan_kernel == 3:
        name += " (+ k_roaring_chunk bitmap build)"
    if scan_kernel == 14:
        name = "k_agg_sparse<containers> (no bitmap build)"
    if scan_kernel == 15:
        name = "k_group_sparse<containers> (chunk bitmaps built in LDS)"
    return name


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def m_dictionary():
    rng = np.random.default_rng(0xC003)
    return np.sort(rng.choice(1 << 20, 65536, replace=False)).astype(np.int32)


def make_segment_buffers(seg_index, rows, seed, cols):
    from pinot_amd.segment import ColumnBuffers, SegmentBuffers, encode_dictionary, fixed_bit_pack
    rng = np.random.default_rng([seed, seg_index])
    seg = SegmentBuffers(f"t_{seed}_{seg_index}", rows)
    mdict = m_dictionary()
    for name, (card, bits) in cols.items():
        ids = rng.integers(0, card, rows, dtype=np.int32)
        dictionary = mdict if name == "m" else np.arange(card, dtype=np.int32)
        dbytes, width = encode_dictionary(dictionary, "INT")
        seg.columns[name] = ColumnBuffers(name, "INT", card, bits, False, fixed_bit_pack(ids, bits), dbytes, width,
                                          dictionary)
    return seg


def built_workload(kind):
    """(query, builder) of a BUILT workload; builder(i, rows) -> (SegmentBuffers, algorithmic bytes of one query
    over that segment, oracle segment of the same values).  config1: the streams the scan reads, over the sorted range's docs only (accountId filter
    ids, day keys, clicks / impressions values).  config5: SURVEY 8(d)'s figure -- the u stream in full plus the
    roaring bytes of the IN list's bitmaps."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    from pinot_amd.segment import create_segment
    from tests import workloads as W
    if kind == "ads":
        def build(i, rows):
            cols = W.ads_columns(rows, seed=0xAD01 + i)
            seg = create_segment(f"ads_{i}", cols)
            days = cols["daysSinceEpoch"][0]
            docs = int(np.count_nonzero((days >= 17849) & (days <= 17856)))
            bits = sum(seg.columns[c].bits for c in ("accountId", "daysSinceEpoch", "clicks", "impressions"))
            return seg, (docs * bits + 7) // 8, lambda: O.build_segment(f"ads_{i}", cols)
        return W.ADS_SQL, build
    ids = list(range(3, 1000, 100))

    def build(i, rows):
        cols = W.hll_columns(rows, seed=0xC005 + i)
        seg = create_segment(f"hll_{i}", cols, inverted=("c",))
        c = seg.columns["c"]
        offs = np.frombuffer(np.ascontiguousarray(c.inverted_index).tobytes()[:4 * (c.cardinality + 1)], ">u4")
        roaring = sum(int(offs[k + 1]) - int(offs[k]) for k in ids if k < c.cardinality)
        return seg, (rows * seg.columns["u"].bits + 7) // 8 + roaring, lambda: O.build_segment(f"hll_{i}", cols)
    return W.hll_sql(ids), build


def algorithmic_bytes(rows_per_seg, nseg, cols):
    return nseg * sum((rows_per_seg * b + 7) // 8 for _, b in cols.values())


def oracle_segments(bufs):
    from oracle import oracle as O
    return [O.segment_from_dict_ids(b.name, {c: dict(dictionary=cb.dictionary_values, fwd=cb.forward_index,
                                                     bits=cb.bits, data_type=cb.data_type, num_docs=b.num_docs)
                                           for c, cb in b.columns.items()}) for b in bufs]


def query_columns(q):
    cols = list(q.group_by)
    for a in q.aggregations:
        cols += a.columns()
    if q.filter is not None:
        cols += q.filter.columns()
    return list(dict.fromkeys(cols))


def flight_main(args, world, rank, dist, device):
    """config4: every step runs the 13 SSB queries over the whole table (one launch set per query); value = rows
    scanned per second summed over the flight (13 x table rows / flight time)."""
    import torch
    from oracle import oracle as O
    from pinot_amd.distributed import DistributedQuery
    from pinot_amd.engine import GpuContext
    from pinot_amd.query import parse_sql
    from pinot_amd.reduce import reduce_groups
    from tests import workloads as W
    distinct, rows_default, seg_default, wdesc = FLIGHTS[args.workload]
    queries = [parse_sql(sql) for sql in W.SSB_QUERIES.values()]
    rows_total = args.rows or rows_default
    nseg = max(1, rows_total // (args.segment_rows or seg_default))
    seg_rows = rows_total // nseg
    mine = [i for i in range(nseg) if i % world == rank]
    t0 = time.time()
    inverted = () if args.workload.endswith("-scan") else W.SSB_INVERTED
    built = {j: W.ssb_segment_buffers(f"ssb_{j}", seg_rows, seed=0xC004 + j, inverted=inverted)
             for j in range(min(distinct, nseg))}
    log(f"[rank {rank}] built {len(built)} distinct segments ({time.time() - t0:.1f}s)")
    ctx = GpuContext(device)
    pinned = [ctx.pin(built[i % distinct]) for i in mine]
    bufs = [built[i % distinct] for i in mine]
    any_buf = built[0]
    for g in dict.fromkeys(g for q in queries for g in q.group_by):  # table-level dictionaries for dense partials
        vals = np.unique(np.concatenate([b.columns[g].dictionary_values for b in built.values()]))
        ctx.set_table_dictionary(g, any_buf.columns[g].data_type, vals)
    ctx.set_schema({c: cb.data_type for c, cb in any_buf.columns.items()})
    runner = DistributedQuery(ctx)
    alg = sum(sum((seg_rows * any_buf.columns[c].bits + 7) // 8 for c in query_columns(q)) * len(mine)
              for q in queries)

    def step():
        ms = 0.0
        for q in queries:
            if world > 1:
                _, _, scan = runner.execute(q, pinned, copy=False)
                ms += scan.device_ms
            else:
                ms += ctx.execute(q, pinned, copy=False).stats.device_ms
        return ms
    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dev_ms = []
    ts = time.perf_counter()
    for _ in range(args.steps):
        dev_ms.append(step())
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - ts
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    total_rows = nseg * seg_rows
    kernel_ms = float(np.mean(dev_ms))
    achieved = alg / (kernel_ms / 1000.0) / 1e9 if kernel_ms > 0 else None
    traffic = load_traffic(args.workload, 1) if world == 1 else None
    moved_gbs = (traffic / (kernel_ms / 1000.0) / 1e9) if traffic and kernel_ms else None
    result = {
        "metric": "filter+group-by rows/s and achieved HBM GB/s, 1B rows",
        "value": len(queries) * total_rows / (ms_per_step / 1000.0), "unit": "rows/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int64",
        "data": (f"synthetic (tests/workloads.py ssb_segment_buffers, {len(built)} distinct {seg_rows}-doc segments "
                 f"pinned as {nseg} segments, sharded over {world} GPU(s))"),
        "config": {"workload": wdesc, "table_rows": total_rows, "segments": nseg, "segments_per_gpu": len(mine),
                   "queries_per_step": len(queries),
                   "parallelism": f"segments sharded x{world}" + (", RCCL reduce-scatter by key range" if world > 1
                                                                  else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                     # the step's PMC FETCH + WRITE bytes (profiles/<round>_pmc_<workload>.json) over the same
                     # device time: the fraction of peak the sparse kernels actually MOVE (frac divides full-column
                     # bytes, most of which the gathers never touch)
                     "achieved_traffic_gbs": moved_gbs,
                     "frac_moved": (moved_gbs / HBM_PEAK_GBS) if moved_gbs else None,
                     "kernel": "13 SSB queries (k_agg_sparse for Q1.x, k_group_sparse for Q2.x-Q4.x, leaves from "
                               "inverted bitmaps or register-direct scans; bytes = the queries' full column bytes, "
                               "which the sparse gathers touch only in part)",
                     "kernel_ms": kernel_ms,
                     "algorithmic_bytes_per_launch": alg},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = host_threads()
        osegs = oracle_segments([built[0]])
        t1 = time.perf_counter()
        exp = [O.execute(q, osegs, 1, filter_stats=False) for q in queries]  # one segment, one thread, every query
        dt1 = time.perf_counter() - t1
        # one segment per thread (the oracle's flight does not scale past one wave of segments: r3 measured 77 s
        # for 39 segments on 16 threads against 2.0 s for one segment on one)
        n = int(max(1, min(len(bufs), threads)))
        sample = oracle_segments(bufs[:n])
        t2 = time.perf_counter()
        for q in queries:
            O.execute(q, sample, threads, filter_stats=False)
        dt = time.perf_counter() - t2
        result["cpu_baseline"] = {
            "value": len(queries) * n * seg_rows / dt, "unit": "rows/s", "cores": threads, "kind": "port",
            "value_t1": len(queries) * seg_rows / dt1, "host_cores": os.cpu_count(), "cpu_model": cpu_model(),
            "cores_note": CPU_NOTE,
            "sample": f"the 13 queries over {n} of {nseg} segments x {seg_rows} rows, oracle C restatement on "
                      f"{threads} host threads, {dt:.2f}s; value_t1 = one segment on one thread, {dt1:.2f}s"}
        if not args.no_parity:  # every query of the flight on one segment, bit-exact (SUM of integer expressions)
            ok = True
            for q, e in zip(queries, exp):
                r = ctx.execute(q, pinned[:1])
                ok = ok and reduce_groups(q, r.keys, r.aggs).rows == reduce_groups(q, e.keys, e.aggs).rows
            result["parity_sample"] = {"segments": 1, "queries": len(queries), "bit_exact": bool(ok)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def host_threads():
    """Host cores this process may use: the affinity mask, capped by OMP_NUM_THREADS (the GPU box sets it to
    the job's CPU share; nproc there reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(bufs, q, threads, target_s=10.0, makers=None):
    """The oracle (C restatement of the reference loop nest, one worker per segment on `threads` host threads,
    as GroupByCombineOperator) over a bounded sample of the same segments: calibrated on one segment on one
    thread (the T = 1 leg), then as many segments as make ~target_s seconds of CPU work on `threads`."""
    from oracle import oracle as O

    def osegs(k):  # oracle segments of the first k (sorted columns / inverted indexes: from the values)
        if makers:  # one oracle segment per distinct maker (setdefault would build every one eagerly)
            built = {}
            for mk in makers[:k]:
                if id(mk) not in built:
                    built[id(mk)] = mk()
            return [built[id(mk)] for mk in makers[:k]]
        return oracle_segments(bufs[:k])
    dt1, _, _ = O.execute_timed(q, osegs(1), 1)  # one segment on one thread
    waves = max(1, int(target_s / max(dt1, 1e-3)))  # segments per thread in ~target_s
    n = int(max(1, min(len(bufs), waves * threads)))
    segs = osegs(n)
    dt, keys, aggs = O.execute_timed(q, segs, threads)
    return n, dt, dt1, keys, aggs


def load_traffic(workload, kernel_count):
    """HBM bytes per launch from profiles/<round>_pmc_<workload>.json (tools/gpu_pmc.sh), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc_{workload}.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        return float(d["hbm_bytes_per_query"])
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=None, help="table rows (sharded across the GPUs); default 1e9, "
                                                           "config1 1e7")
    ap.add_argument("--segment-rows", type=int, default=None, help="default 1e7")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample size in seconds of work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--workload", default="config3", choices=sorted(list(WORKLOADS) + list(BUILT) + list(FLIGHTS)))
    ap.add_argument("--devices", default=None,
                    help="comma-separated HIP ordinals: ONE process drives one multi-device context over them "
                         "(ph_ctx_create_multi, the Pinot server's drop-in; a repeated ordinal is a logical shard), "
                         "instead of one process per GPU")
    ap.add_argument("--transport", default="peer", choices=["peer", "rccl"], help="with --devices")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        # one process per GPU over RCCL; PH_DIST_BACKEND=gloo rehearses the N > 1 path on a box with fewer GPUs than
        # ranks (ranks share devices round-robin; gloo all-reduces and slices where RCCL reduce-scatters)
        local_rank = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank)
        backend = os.environ.get("PH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    device = local_rank
    if args.workload in FLIGHTS:
        return flight_main(args, world, rank, dist, device)

    from pinot_amd.distributed import DistributedQuery
    from pinot_amd.engine import GpuContext
    from pinot_amd.query import parse_sql

    built = BUILT.get(args.workload)
    if built:
        kind, distinct, rows_default, seg_default, wdesc = built
        query, builder = built_workload(kind)
        cols = None
    else:
        query, cols, wdesc = WORKLOADS[args.workload]
        rows_default, seg_default = 1_000_000_000, 10_000_000
    rows_total = args.rows or rows_default
    q = parse_sql(query)
    nseg = max(1, rows_total // (args.segment_rows or seg_default))
    seg_rows = rows_total // nseg
    mine = [i for i in range(nseg) if i % world == rank]  # this rank's shard of the table
    t0 = time.time()
    devices = [int(x) for x in args.devices.split(",")] if args.devices else None
    if devices and world > 1:
        raise SystemExit("--devices drives every device from one process: run it without torch.distributed")
    ctx = GpuContext(device) if not devices else GpuContext(devices=devices, transport=args.transport)
    bufs, pinned, seg_alg, ora_makers = [], [], [], []
    distinct_bufs = {}
    for k, i in enumerate(mine):
        if built:  # `distinct` different segments, each pinned as many times as the table needs
            if i % distinct not in distinct_bufs:
                distinct_bufs[i % distinct] = builder(i % distinct, seg_rows)
            b, a, mk = distinct_bufs[i % distinct]
            seg_alg.append(a)
            ora_makers.append(mk)
        else:
            b = make_segment_buffers(i, seg_rows, seed=1000, cols=cols)
        # DISTINCTCOUNTHLL columns get their HLL tables at pin (ph_column_desc.hll_log2m), not in the first query
        pinned.append(ctx.pin(b, hll_columns=[a.column for a in q.aggregations if a.function == "DISTINCTCOUNTHLL"]))
        bufs.append(b)
        if k % 20 == 19:
            log(f"[rank {rank}] pinned {k + 1}/{len(mine)} segments ({time.time() - t0:.1f}s)")
    # table-level dictionaries: identical on every rank, so dense group ids line up for the RCCL merge
    if built:
        # every rank builds the same distinct segments' dictionaries (deterministic seeds)
        for g in q.group_by:
            vals = set()
            for j in range(min(distinct, nseg)):
                vals.update((distinct_bufs.get(j) or builder(j, seg_rows))[0].columns[g].dictionary_values.tolist())
            ctx.set_table_dictionary(g, "INT", np.array(sorted(vals), dtype=np.int32))
        ctx.set_schema({c: "INT" for c in (bufs[0].columns if bufs else {})})
    else:
        for g in q.group_by:
            ctx.set_table_dictionary(g, "INT", np.arange(cols[g][0], dtype=np.int32))
        ctx.set_schema({c: "INT" for c in cols})  # a rank without segments still builds the common dense layout

    runner = DistributedQuery(ctx)
    last = {}

    def step():
        if world > 1:
            res, shard, scan = runner.execute(q, pinned, copy=False)
            last["res"], last["shard"] = res, shard
            return scan.device_ms, scan.plan_mode
        r = ctx.execute(q, pinned, copy=False)
        last["res"] = r
        last["kernel"] = r.stats.scan_kernel
        if devices:
            # the call's wall time split into its phases (scan / merge / finalize wall times, and the rest: planning,
            # layout and result assembly on the host); scan_device = the longest device's scan kernels
            phases.append({"scan": r.stats.scan_ms, "scan_device": r.stats.device_ms, "merge": r.stats.merge_ms,
                           "finalize": r.stats.finalize_ms,
                           "host": r.stats.host_ms - r.stats.scan_ms - r.stats.merge_ms - r.stats.finalize_ms,
                           "call": r.stats.host_ms, "devices": r.stats.num_devices})
        return r.stats.device_ms, r.stats.mode

    phases = []
    log(f"[rank {rank}] pinned {len(pinned)} segments ({time.time() - t0:.1f}s); warmup")
    for _ in range(args.warmup):
        step()
    phases.clear()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    log(f"[rank {rank}] timing {args.steps} steps")
    dev_ms = []
    mode = -1
    ts = time.perf_counter()
    for _ in range(args.steps):
        ms, mode = step()
        dev_ms.append(ms)
        if world > 1:
            phases.append(dict(runner.last_times))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - ts
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    total_rows = nseg * seg_rows
    value = total_rows / (ms_per_step / 1000.0)
    # roofline of the dominant kernel: this rank's scan kernels (HIP events on their stream) over this rank's
    # algorithmic bytes
    kernel_ms = float(np.mean(dev_ms)) if dev_ms else 0.0
    alg = sum(seg_alg) if built else algorithmic_bytes(seg_rows, len(mine), cols)
    achieved = alg / (kernel_ms / 1000.0) / 1e9 if kernel_ms > 0 else None
    traffic = load_traffic(args.workload, 1) if world == 1 else None

    result = {
        "metric": "filter+group-by rows/s and achieved HBM GB/s, 1B rows",
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": (f"synthetic (seeded PCG64 dictIds, one {total_rows}-row table of {nseg} x {seg_rows}-doc segments, "
                 f"sharded over {world} GPU(s))" if not built else
                 f"synthetic (tests/workloads.py generators, {min(built[1], nseg)} distinct {seg_rows}-doc segments "
                 f"pinned as {nseg} segments, sharded over {world} GPU(s))"),
        "config": {"workload": wdesc, "table_rows": total_rows, "segments": nseg, "segments_per_gpu": len(mine),
                   "parallelism": (f"one process, multi-device context over ordinals {devices} (segments placed by "
                                   f"rows, dense partials reduce-scattered by key shard, {args.transport} transport)"
                                   if devices else
                                   f"segments sharded x{world}" + (", RCCL reduce-scatter by key range" if world > 1
                                                                   else ""))},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                     "kernel": kernel_name(mode, last.get("kernel", 1)), "kernel_ms": kernel_ms,
                     "algorithmic_bytes_per_launch": alg,
                     # bytes the kernels actually moved (PMC FETCH + WRITE, profiles/) over the same device time
                     "achieved_traffic_gbs": (traffic / (kernel_ms / 1000.0) / 1e9) if traffic and kernel_ms else None,
                     "frac_moved": (traffic / (kernel_ms / 1000.0) / 1e9 / HBM_PEAK_GBS) if traffic and kernel_ms
                     else None},
    }
    if phases:
        result["phases_ms"] = {k: float(np.mean([p[k] for p in phases])) for k in phases[0]}
    if last.get("res") is not None:
        result["groups"] = last["res"].num_groups
    if devices:
        result["n_gpus"] = len(set(devices))
        result["devices"] = devices
    if rank == 0 and world == 1 and not args.no_cpu and not devices:
        threads = host_threads()
        log(f"[rank {rank}] {ms_per_step:.3f} ms/step; CPU baseline on {threads} threads")
        n, dt, dt1, keys, aggs = cpu_baseline(bufs, q, threads, args.cpu_seconds, ora_makers or None)
        rows = n * seg_rows
        result["cpu_baseline"] = {"value": rows / dt, "unit": "rows/s", "cores": threads, "kind": "port",
                                  "value_t1": seg_rows / dt1, "host_cores": os.cpu_count(),
                                  "cpu_model": cpu_model(), "cores_note": CPU_NOTE,
                                  "sample": f"{n} of {nseg} segments x {seg_rows} rows (same data and query), oracle "
                                            f"C restatement of the reference loop nest (one worker per segment, as "
                                            f"GroupByCombineOperator) on {threads} host threads, {dt:.2f}s; "
                                            f"value_t1 = one segment on one thread, {dt1:.2f}s"}
        if not args.no_parity and built:
            # parity on the sample: the GPU's reduced rows vs the oracle's (all columns bit-exact; HLL registers
            # compared raw)
            from oracle import oracle as O
            from pinot_amd.reduce import reduce_groups
            r = ctx.execute(q, pinned[:n])
            built_o = {}
            for mk in ora_makers[:n]:
                if id(mk) not in built_o:
                    built_o[id(mk)] = mk()
            e = O.execute(q, [built_o[id(mk)] for mk in ora_makers[:n]], filter_stats=False)
            ok = reduce_groups(q, r.keys, r.aggs).rows == reduce_groups(q, e.keys, e.aggs).rows
            for k, a in enumerate(q.aggregations):
                if a.function == "DISTINCTCOUNTHLL":
                    ok = ok and all(np.array_equal(x[k], y[k]) for x, y in zip(r.aggs, e.aggs))
            result["parity_sample"] = {"segments": n, "groups": int(r.num_groups), "bit_exact": bool(ok)}
        elif not args.no_parity:
            # parity on the sample: GPU over the same segments vs the oracle -- group keys, COUNT, integer SUM,
            # MIN, MAX bit-exact (synthetic group dictionaries are 0..C-1, so value == global id)
            r = ctx.execute(q, pinned[:n])
            order = np.argsort(keys)
            k_cpu = keys[order]
            a_cpu = aggs[order]
            k_gpu = np.zeros(r.num_groups, np.uint64)
            stride = 1
            for gi, g in enumerate(q.group_by):
                k_gpu += r.key_columns[gi].astype(np.uint64) * np.uint64(stride)
                stride *= cols[g][0]
            og = np.argsort(k_gpu)
            a_gpu = np.stack([c.astype(np.float64) for c in r.agg_columns], axis=1)[og]
            ok = bool(np.array_equal(k_gpu[og], k_cpu) and np.array_equal(a_gpu, a_cpu))
            result["parity_sample"] = {"segments": n, "groups": int(len(k_cpu)), "bit_exact": ok}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
