"""Broker-side reduce for the filter -> aggregation / group-by path.

Mirrors the final steps the reference applies after the server-side combine:

* ``AggregationFunction.extractFinalResult`` -- COUNT -> long, SUM/MIN/MAX -> double,
  DISTINCTCOUNTHLL -> ``HyperLogLog.cardinality()`` (DistinctCountHLLAggregationFunction.java:362-364).
* ``IndexedTable.finish`` / ``GroupByDataTableReducer.reduceAndSetResults`` -- ORDER BY over group-by
  columns and aggregations (ASC/DESC), then LIMIT (core/data/table/IndexedTable.java:148-173,
  core/query/reduce/GroupByDataTableReducer.java:99).
* Aggregation-only queries produce exactly one row (AggregationDataTableReducer).

A group-by query without ORDER BY returns an arbitrary subset in the reference; here groups are
returned in key order so results are deterministic.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, List, Sequence

import numpy as np

from .query import COUNT, DISTINCTCOUNTHLL, MAX, MIN, SUM, QueryContext


def _java_round(x: float) -> int:
    if math.isnan(x):
        return 0
    if math.isinf(x):
        return (1 << 63) - 1 if x > 0 else -(1 << 63)
    return int(math.floor(x + 0.5))


def hll_cardinality(registers: np.ndarray, log2m: int) -> int:
    """clearspring HyperLogLog.cardinality() (stream 2.7.0) over raw 1-byte registers."""
    m = 1 << log2m
    reg = np.asarray(registers, dtype=np.int64)
    assert reg.shape[-1] == m
    s = float(np.sum(1.0 / np.left_shift(np.int64(1), reg).astype(np.float64)))
    zeros = float(np.sum(reg == 0))
    if log2m == 4:
        alpha_mm = 0.673 * m * m
    elif log2m == 5:
        alpha_mm = 0.697 * m * m
    elif log2m == 6:
        alpha_mm = 0.709 * m * m
    else:
        alpha_mm = (0.7213 / (1 + 1.079 / m)) * m * m
    estimate = alpha_mm * (1 / s)
    if estimate <= (5.0 / 2.0) * m:
        return _java_round(m * math.log(m / zeros)) if zeros > 0 else (1 << 63) - 1
    return _java_round(estimate)


def hll_serialize(registers: np.ndarray, log2m: int) -> bytes:
    """ObjectSerDeUtils HyperLogLog serializer: int32 BE log2m, int32 BE byte size, then the clearspring
    RegisterSet words (6 x 5-bit registers per int, register i at word i/6, shift 5*(i%6)), BE
    (ObjectSerDeUtils.java:535-560, HyperLogLogUtils.java:28-43)."""
    m = 1 << log2m
    nwords = m // 6 + 1
    words = np.zeros(nwords, dtype=np.uint32)
    for i in range(m):
        words[i // 6] |= np.uint32(int(registers[i]) & 0x1F) << np.uint32(5 * (i % 6))
    return (np.array([log2m, 4 * nwords], dtype=">i4").tobytes() + words.astype(">u4").tobytes())


@dataclass
class ResultTable:
    columns: List[str]
    rows: List[List[Any]]

    def __repr__(self):
        return f"ResultTable({self.columns}, {self.rows[:5]}{'...' if len(self.rows) > 5 else ''})"


def final_value(spec, value):
    if spec.function == COUNT:
        return int(value)
    if spec.function == DISTINCTCOUNTHLL:
        return hll_cardinality(value, spec.log2m)
    return float(value)


def reduce_groups(q: QueryContext, keys: Sequence[tuple], aggs: Sequence[Sequence[Any]]) -> ResultTable:
    """keys[i]: tuple of group-by values of group i; aggs[i][k]: intermediate result of
    aggregation k (COUNT int, SUM/MIN/MAX float, HLL register array)."""
    finals = [[final_value(q.aggregations[k], a[k]) for k in range(len(q.aggregations))] for a in aggs]
    idx = list(range(len(keys)))
    if q.group_by:
        # deterministic base order: keys ascending
        idx.sort(key=lambda i: keys[i])
        for ob in reversed(q.order_by):
            if ob.kind == "column":
                c = q.group_by.index(ob.ref)
                idx.sort(key=lambda i, c=c: keys[i][c], reverse=not ob.asc)
            else:
                idx.sort(key=lambda i, k=ob.ref: finals[i][k], reverse=not ob.asc)
        idx = idx[: q.limit]
    rows = []
    for i in idx:
        row = []
        for s in q.select:
            if s.kind == "column":
                row.append(keys[i][q.group_by.index(s.ref)])
            else:
                row.append(finals[i][s.ref])
        rows.append(row)
    return ResultTable(q.result_columns(), rows)
