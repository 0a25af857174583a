"""Generate the golden fixtures under tests/golden/ from the reference's own test data.

Run in the build container (needs /root/reference); the outputs are committed so the
GPU box (which has no /root/reference) never reads the reference.

Outputs
-------
test_data_sv.npz
    The 11 columns that ``BaseSingleValueQueriesTest`` (pinot-core/src/test/java/org/apache/pinot/
    queries/BaseSingleValueQueriesTest.java:54-68,99-107) selects from
    ``pinot-core/src/test/resources/data/test_data-sv.avro`` (30 000 records). Data only:
    INT columns as int32 arrays, STRING columns as numpy unicode arrays.

The Avro container file is parsed by a minimal reader written here (null codec, union
["null", T] fields of int/string/long/float/double), following the public Avro 1.x
specification (zig-zag varints, length-prefixed strings, sync-marker blocks).
"""
import json
import os
import sys

import numpy as np

REF_AVRO = "/root/reference/pinot-core/src/test/resources/data/test_data-sv.avro"
HERE = os.path.dirname(os.path.abspath(__file__))

# BaseSingleValueQueriesTest.java:99-107 (schema) -- column -> (Pinot data type, field type)
KAT_COLUMNS = {
    "column1": "INT", "column3": "INT", "column5": "STRING", "column6": "INT",
    "column7": "INT", "column9": "INT", "column11": "STRING", "column12": "STRING",
    "column17": "INT", "column18": "INT", "daysSinceEpoch": "INT",
}
# Pinot default null values (FieldSpec.java: DEFAULT_DIMENSION_NULL_VALUE_OF_INT = Integer.MIN_VALUE,
# DEFAULT_METRIC_NULL_VALUE_OF_INT = 0, DEFAULT_DIMENSION_NULL_VALUE_OF_STRING = "null").
METRICS = {"column1", "column3", "column17", "column18"}


class _Reader:
    def __init__(self, buf):
        self.b = buf
        self.p = 0

    def long(self):
        shift = 0
        acc = 0
        while True:
            c = self.b[self.p]
            self.p += 1
            acc |= (c & 0x7F) << shift
            if not (c & 0x80):
                break
            shift += 7
        return (acc >> 1) ^ -(acc & 1)

    def bytes_(self):
        n = self.long()
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def raw(self, n):
        v = self.b[self.p:self.p + n]
        self.p += n
        return v


def read_avro(path):
    data = open(path, "rb").read()
    r = _Reader(data)
    assert r.raw(4) == b"Obj\x01", "not an Avro object container"
    meta = {}
    while True:
        n = r.long()
        if n == 0:
            break
        if n < 0:
            r.long()
            n = -n
        for _ in range(n):
            k = r.bytes_().decode()
            meta[k] = r.bytes_()
    codec = meta.get("avro.codec", b"null").decode()
    assert codec == "null", codec
    schema = json.loads(meta["avro.schema"])
    sync = r.raw(16)
    fields = []
    for f in schema["fields"]:
        t = f["type"]
        if isinstance(t, list):
            assert t[0] == "null" and len(t) == 2, t
            fields.append((f["name"], t[1], True))
        else:
            fields.append((f["name"], t, False))
    cols = {name: [] for name, _, _ in fields}
    while r.p < len(data):
        count = r.long()
        _size = r.long()
        for _ in range(count):
            for name, typ, nullable in fields:
                if nullable and r.long() == 0:
                    cols[name].append(None)
                    continue
                if typ in ("int", "long"):
                    cols[name].append(r.long())
                elif typ == "string":
                    cols[name].append(r.bytes_().decode("utf-8"))
                elif typ == "float":
                    cols[name].append(float(np.frombuffer(r.raw(4), "<f4")[0]))
                elif typ == "double":
                    cols[name].append(float(np.frombuffer(r.raw(8), "<f8")[0]))
                else:
                    raise ValueError(typ)
        assert r.raw(16) == sync
    return cols


def main():
    if not os.path.exists(REF_AVRO):
        sys.exit("reference test data not present; fixtures are already committed")
    cols = read_avro(REF_AVRO)
    out = {}
    for c, dt in KAT_COLUMNS.items():
        vals = cols[c]
        nulls = sum(v is None for v in vals)
        if dt == "INT":
            fill = 0 if c in METRICS else -(2 ** 31)
            out[c] = np.array([fill if v is None else v for v in vals], dtype=np.int32)
        else:
            out[c] = np.array(["null" if v is None else v for v in vals])
        print(f"{c:16s} {dt:6s} rows={len(vals)} nulls={nulls} card={len(np.unique(out[c]))}")
    np.savez_compressed(os.path.join(HERE, "test_data_sv.npz"), **out)


if __name__ == "__main__":
    main()
