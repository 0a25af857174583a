"""The boundary's threading and interruption contract (SURVEY.md 8(b) Threading, 5 Failure detection):

* concurrent calls on ONE context from several host threads (Pinot runs queries on executor worker threads,
  BaseCombineOperator.java:96-141) -- each call takes its own stream / events / scratch, and every result equals
  the oracle's;
* interruption: ph_query.interrupt set before or during a call, and an end time already passed (QueryContext
  timeoutMs), return PH_ERR_CANCELLED (BaseOperator.java:39, GroupByCombineOperator.java:225-234); the context
  keeps working afterwards.
"""
import ctypes
import threading

import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.native import CancelledError
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment

pytestmark = pytest.mark.gpu

QUERIES = [
    "SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE f BETWEEN 100 AND 599",
    "SELECT a, COUNT(*), SUM(m) FROM t WHERE f < 300 GROUP BY a ORDER BY a LIMIT 1000",
    "SET numGroupsLimit=2000000; SELECT a, b, SUM(m), COUNT(*), MAX(m) FROM t GROUP BY a, b ORDER BY a, b "
    "LIMIT 2000000",
    "SELECT DISTINCTCOUNTHLL(m) FROM t WHERE a IN (1, 7, 30)",
    "SELECT a, SUM(m - f), MIN(m * f) FROM t WHERE b <> 3 GROUP BY a ORDER BY a LIMIT 1000",
]


def _tables():
    rng = np.random.default_rng(77)
    out = []
    for n in (300_000, 200_017):
        out.append({"a": (rng.integers(0, 60, n).astype(np.int32), "INT"),
                    "b": (rng.integers(0, 2000, n).astype(np.int32), "INT"),
                    "f": (rng.integers(0, 1000, n).astype(np.int32), "INT"),
                    "m": (rng.integers(-5000, 1 << 20, n).astype(np.int32), "INT")})
    return out


@pytest.fixture(scope="module")
def setup():
    from pinot_amd.engine import GpuContext
    ctx = GpuContext(0)
    tables = _tables()
    gpu = [ctx.pin(create_segment(f"c{i}", t, inverted=("a",))) for i, t in enumerate(tables)]
    ora = [O.build_segment(f"c{i}", t, inverted=("a",)) for i, t in enumerate(tables)]
    expected = {}
    for sql in QUERIES:
        q = parse_sql(sql)
        e = O.execute(q, ora)
        expected[sql] = reduce_groups(q, e.keys, e.aggs).rows
    yield ctx, gpu, expected
    ctx.close()


def test_concurrent_queries_one_context(setup):
    ctx, gpu, expected = setup
    errors = []

    def worker(k):
        try:
            for it in range(6):
                sql = QUERIES[(k + it) % len(QUERIES)]
                q = parse_sql(sql)
                r = ctx.execute(q, gpu)
                got = reduce_groups(q, r.keys, r.aggs).rows
                if got != expected[sql]:
                    errors.append((k, it, sql))
        except Exception as e:  # noqa: BLE001 -- surfaced below
            errors.append((k, repr(e)))

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a query thread did not finish"
    assert errors == []


def test_interrupt_before_and_deadline(setup):
    ctx, gpu, expected = setup
    q = parse_sql(QUERIES[0])
    flag = ctypes.c_int32(1)
    with pytest.raises(CancelledError):
        ctx.execute(q, gpu, interrupt=flag)
    late = parse_sql("SET timeoutMs=-1; " + QUERIES[2])
    with pytest.raises(CancelledError):
        ctx.execute(late, gpu)
    # the context is intact afterwards; an interruptible call that is not interrupted returns the full answer
    flag.value = 0
    r = ctx.execute(parse_sql(QUERIES[1]), gpu, interrupt=flag)
    assert reduce_groups(parse_sql(QUERIES[1]), r.keys, r.aggs).rows == expected[QUERIES[1]]
    r = ctx.execute(parse_sql("SET timeoutMs=60000; " + QUERIES[0]), gpu)
    assert reduce_groups(q, r.keys, r.aggs).rows == expected[QUERIES[0]]


def test_interrupt_during_long_scan(setup, monkeypatch):
    # an interruptible scan checks between batches; with one chunk (16384 docs) per batch (PH_INTERRUPT_CHUNKS)
    # a ~1.3G-doc scan takes seconds, so a flag set 50 ms after the start lands mid-scan
    import time
    ctx, gpu, _ = setup
    monkeypatch.setenv("PH_INTERRUPT_CHUNKS", "1")
    flag = ctypes.c_int32(0)
    big = gpu * 2600
    q = parse_sql("SELECT COUNT(*), SUM(m) FROM t WHERE f BETWEEN 10 AND 900")
    timer = threading.Timer(0.05, lambda: setattr(flag, "value", 1))
    timer.start()
    t0 = time.perf_counter()
    with pytest.raises(CancelledError):
        ctx.execute(q, big, interrupt=flag)
    timer.join()
    assert time.perf_counter() - t0 < 30


def test_first_queries_after_pin_run_concurrently(setup):
    # the derived streams are built at pin (ph_segment_pin: the INT value streams, and the HLL table requested by
    # hll_columns), so the first queries on fresh segments share nothing to build: four threads start their first
    # query together on newly pinned segments, each result equals the oracle's, and the segments' device bytes
    # already include the value streams and the HLL table before any query ran
    ctx, _, expected = setup
    tables = _tables()
    fresh = [ctx.pin(create_segment(f"f{i}", t, inverted=("a",)), hll_columns=("m",)) for i, t in enumerate(tables)]
    plain = [ctx.pin(create_segment(f"p{i}", t, inverted=("a",))) for i, t in enumerate(tables)]
    for f, p in zip(fresh, plain):
        assert f.device_bytes > p.device_bytes  # + the HLL table (4 B per dictId), built at pin
    before = [f.device_bytes for f in fresh]
    errors = []
    start = threading.Barrier(4)

    def worker(k):
        try:
            start.wait()
            sql = QUERIES[[0, 3, 4, 3][k]]
            q = parse_sql(sql)
            r = ctx.execute(q, fresh)
            if reduce_groups(q, r.keys, r.aggs).rows != expected[sql]:
                errors.append((k, sql))
        except Exception as e:  # noqa: BLE001 -- surfaced below
            errors.append((k, repr(e)))

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a query thread did not finish"
    assert errors == []
    assert [f.device_bytes for f in fresh] == before  # no query derived anything more for these columns' aggregates
