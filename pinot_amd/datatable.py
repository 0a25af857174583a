"""Broker side of the server -> broker DataTable V4.

``decode`` reads the bytes ``ph_result_datatable`` / ``GpuContext.execute_datatable`` produce, exactly as
``DataTableImplV4(ByteBuffer)`` does (pinot-common/.../datatable/DataTableImplV4.java: header, exceptions, string
dictionary, DataSchema.fromBytes, fixed-size rows, variable-size data, metadata by MetadataKey id).
``reduce_datatables`` is the broker's merge of several servers' tables for this path:
GroupByDataTableReducer.reduceAndSetResults (core/query/reduce/GroupByDataTableReducer.java:99) /
AggregationDataTableReducer -- intermediate results merged per group key with AggregationFunction.merge
(COUNT / SUM add, MIN / MAX, DISTINCTCOUNTHLL HyperLogLog.addAll = register max), then the final results, ORDER BY
and LIMIT (pinot_amd.reduce.reduce_groups).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, Sequence

import numpy as np

from .query import COUNT, DISTINCTCOUNTHLL, MAX, MIN, SUM, QueryContext
from .reduce import ResultTable, reduce_groups

# MetadataKey id -> (name, value type) (DataTable.java:103-137); "I" int, "L" long, "S" string
METADATA_KEYS = {1: ("table", "S"), 2: ("numDocsScanned", "L"), 3: ("numEntriesScannedInFilter", "L"),
                 4: ("numEntriesScannedPostFilter", "L"), 5: ("numSegmentsQueried", "I"),
                 6: ("numSegmentsProcessed", "I"), 7: ("numSegmentsMatched", "I"),
                 8: ("numConsumingSegmentsQueried", "I"), 9: ("minConsumingFreshnessTimeMs", "L"),
                 10: ("totalDocs", "L"), 11: ("numGroupsLimitReached", "S"), 12: ("timeUsedMs", "L"),
                 13: ("traceInfo", "S"), 14: ("requestId", "L"), 15: ("numResizes", "I"), 16: ("resizeTimeMs", "L"),
                 17: ("threadCpuTimeNs", "L"), 18: ("systemActivitiesCpuTimeNs", "L"),
                 19: ("responseSerializationCpuTimeNs", "L"), 20: ("numSegmentsPrunedByServer", "I"),
                 21: ("numSegmentsPrunedByInvalid", "I"), 22: ("numSegmentsPrunedByLimit", "I"),
                 23: ("numSegmentsPrunedByValue", "I"), 24: ("explainPlanNumEmptyFilterSegments", "I"),
                 25: ("explainPlanNumMatchAllFilterSegments", "I"), 26: ("numConsumingSegmentsProcessed", "I"),
                 27: ("numConsumingSegmentsMatched", "I"), 28: ("numBlocks", "I"), 29: ("numRows", "I"),
                 30: ("operatorExecutionTimeMs", "L"), 31: ("operatorId", "S"), 32: ("operatorExecStartTimeMs", "L"),
                 33: ("operatorExecEndTimeMs", "L")}
HLL_OBJECT_TYPE = 6  # ObjectSerDeUtils.ObjectType.HyperLogLog


@dataclass
class DataTable:
    column_names: List[str]
    column_types: List[str]
    rows: List[List[Any]]
    metadata: Dict[str, str] = field(default_factory=dict)
    exceptions: Dict[int, str] = field(default_factory=dict)


class _Reader:
    def __init__(self, b: bytes, pos: int = 0):
        self.b, self.p = b, pos

    def i32(self) -> int:
        v = struct.unpack_from(">i", self.b, self.p)[0]
        self.p += 4
        return v

    def i64(self) -> int:
        v = struct.unpack_from(">q", self.b, self.p)[0]
        self.p += 8
        return v

    def string(self) -> str:
        n = self.i32()
        s = self.b[self.p:self.p + n].decode("utf-8")
        self.p += n
        return s


def hll_deserialize(b: bytes):
    """HyperLogLog from ObjectSerDeUtils bytes (int log2m, int byte size, RegisterSet words) -> (log2m, uint8
    registers)."""
    log2m, nbytes = struct.unpack_from(">ii", b, 0)
    words = np.frombuffer(b[8:8 + nbytes], ">u4").astype(np.uint32)
    m = 1 << log2m
    i = np.arange(m)
    regs = (words[i // 6] >> (5 * (i % 6)).astype(np.uint32)) & 0x1F
    return log2m, regs.astype(np.uint8)


def decode(buf: bytes) -> DataTable:
    r = _Reader(buf)
    version = r.i32()
    if version != 4:
        raise ValueError(f"DataTable version {version} (only V4)")
    nrows, ncols = r.i32(), r.i32()
    sec = [(r.i32(), r.i32()) for _ in range(5)]  # exceptions, dictionary, schema, fixed, variable
    exceptions, sdict, names, types = {}, [], [], []
    if sec[0][1]:
        e = _Reader(buf, sec[0][0])
        for _ in range(e.i32()):
            code = e.i32()
            exceptions[code] = e.string()
    if sec[1][1]:
        d = _Reader(buf, sec[1][0])
        sdict = [d.string() for _ in range(d.i32())]
    if sec[2][1]:
        s = _Reader(buf, sec[2][0])
        n = s.i32()
        names = [s.string() for _ in range(n)]
        types = [s.string() for _ in range(n)]
    width = {"INT": 4, "FLOAT": 4, "STRING": 4, "LONG": 8, "DOUBLE": 8}
    offs, row = [], 0
    for t in types:
        offs.append(row)
        row += width.get(t, 8)
    fixed = buf[sec[3][0]:sec[3][0] + sec[3][1]]
    var = buf[sec[4][0]:sec[4][0] + sec[4][1]]
    rows = []
    for i in range(nrows):
        base = i * row
        vals = []
        for c, t in enumerate(types):
            o = base + offs[c]
            if t == "INT":
                vals.append(struct.unpack_from(">i", fixed, o)[0])
            elif t == "LONG":
                vals.append(struct.unpack_from(">q", fixed, o)[0])
            elif t == "FLOAT":
                vals.append(struct.unpack_from(">f", fixed, o)[0])
            elif t == "DOUBLE":
                vals.append(struct.unpack_from(">d", fixed, o)[0])
            elif t == "STRING":
                vals.append(sdict[struct.unpack_from(">i", fixed, o)[0]])
            elif t == "OBJECT":  # CustomObject: (offset, length) -> int type + bytes
                vo, ln = struct.unpack_from(">ii", fixed, o)
                otype = struct.unpack_from(">i", var, vo)[0]
                vals.append((otype, var[vo + 4:vo + 4 + ln]))
            else:
                raise ValueError(f"column type {t}")
        rows.append(vals)
    md = {}
    mr = _Reader(buf, sec[4][0] + sec[4][1])
    if mr.i32():
        for _ in range(mr.i32()):
            key = METADATA_KEYS.get(mr.i32())
            if key is None:
                continue
            name, vt = key
            md[name] = str(mr.i32()) if vt == "I" else (str(mr.i64()) if vt == "L" else mr.string())
    return DataTable(names, types, rows, md, exceptions)


def _merge(fn, a, b):
    if fn in (COUNT, SUM):
        return a + b
    if fn == MIN:
        return min(a, b)
    if fn == MAX:
        return max(a, b)
    return np.maximum(a, b)  # HyperLogLog.addAll


def reduce_datatables(q: QueryContext, tables: Sequence[DataTable]) -> ResultTable:
    """Broker merge of the servers' DataTables for ``q`` (GroupByDataTableReducer / AggregationDataTableReducer)."""
    nk = len(q.group_by)
    groups: Dict[tuple, list] = {}
    for t in tables:
        for row in t.rows:
            key = tuple(row[:nk])
            inter = []
            for k, a in enumerate(q.aggregations):
                v = row[nk + k]
                if a.function == DISTINCTCOUNTHLL:
                    otype, payload = v
                    assert otype == HLL_OBJECT_TYPE
                    v = hll_deserialize(payload)[1]
                inter.append(v)
            if key in groups:
                groups[key] = [_merge(a.function, x, y) for a, x, y in zip(q.aggregations, groups[key], inter)]
            else:
                groups[key] = inter
    if not nk and not groups:
        groups[()] = [0 if a.function == COUNT else None for a in q.aggregations]
    keys = list(groups)
    return reduce_groups(q, keys, [groups[k] for k in keys])
