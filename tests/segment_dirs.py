"""On-disk segment directories for the loader tests (test infrastructure).

* ``write_v3`` / ``write_v1`` lay a SegmentBuffers out the way the reference's segment creator does:
  V3 = ``v3/metadata.properties`` + ``v3/index_map`` + ``v3/columns.psf`` with an 8-byte magic
  0xdeadbeefdeafbead before every buffer, ``size`` counting the magic (SingleFileIndexDirectory.java:72,170-204);
  V1 = one file per index (V1Constants.Indexes / Dict: ``.dict``, ``.sv.unsorted.fwd``, ``.sv.sorted.fwd``,
  ``.sv.raw.fwd``, ``.bitmap.inv``); raw columns carry ``hasDictionary = false`` and only a forward index.  Metadata keys: V1Constants.MetadataKeys, SegmentColumnarIndexCreator.addColumnMetadataInfo.
* ``read_dir`` is an independent reader of either layout that builds the CPU oracle's segment (the checker for
  ph_segment_load_dir).  ``tests/golden/v1_padding*`` are two V1 segments the reference itself wrote
  (pinot-core/src/test/resources/data/padding{Null,Old}.tar.gz).
"""
from __future__ import annotations

import os

import numpy as np

from oracle import oracle as O
from tests import raw_codecs as RC

MAGIC = (0xDEADBEEFDEAFBEAD).to_bytes(8, "big")
_NP = {"INT": ">i4", "LONG": ">i8", "FLOAT": ">f4", "DOUBLE": ">f8"}


def _metadata(seg, extra=None):
    lines = [f"segment.name = {seg.name}", f"segment.total.docs = {seg.num_docs}",
             "segment.padding.character = \\\\u0000"]  # as the reference writes it (creator :424)
    for c, cb in seg.columns.items():
        key = c.replace(":", "\\:").replace("=", "\\=")
        entry = cb.entry_size if cb.data_type == "STRING" else 0
        lines += [f"column.{key}.cardinality = {cb.cardinality}", f"column.{key}.totalDocs = {seg.num_docs}",
                  f"column.{key}.dataType = {cb.data_type}", f"column.{key}.bitsPerElement = {cb.bits}",
                  f"column.{key}.lengthOfEachEntry = {entry}", f"column.{key}.columnType = DIMENSION",
                  f"column.{key}.isSorted = {'true' if cb.is_sorted else 'false'}",
                  f"column.{key}.hasDictionary = {'false' if cb.raw else 'true'}",
                  f"column.{key}.hasInvertedIndex = {'true' if cb.inverted_index is not None else 'false'}",
                  f"column.{key}.isSingleValues = true"]
    for k, v in (extra or {}).items():
        lines.append(f"{k} = {v}")
    return "# segment metadata\n" + "\n".join(lines) + "\n"


def _buffers(cb):
    ri = [("range_index", np.ascontiguousarray(cb.range_index).tobytes())] if cb.range_index is not None else []
    if cb.raw:  # no-dictionary column: the raw chunk forward index (+ a range index)
        return [("forward_index", np.ascontiguousarray(cb.forward_index).tobytes())] + ri
    out = [("dictionary", np.ascontiguousarray(cb.dictionary).tobytes()),
           ("forward_index", np.ascontiguousarray(cb.forward_index).tobytes())]
    if cb.inverted_index is not None:
        out.append(("inverted_index", np.ascontiguousarray(cb.inverted_index).tobytes()))
    return out + ri


def write_v3(seg, path, extra_meta=None):
    d = os.path.join(path, "v3")
    os.makedirs(d, exist_ok=True)
    index_map, blob, off = [], bytearray(), 0
    for c in sorted(seg.columns):
        for idx, payload in _buffers(seg.columns[c]):
            entry = MAGIC + payload
            index_map += [f"{c}.{idx}.startOffset = {off}", f"{c}.{idx}.size = {len(entry)}"]
            blob += entry
            off += len(entry)
    open(os.path.join(d, "metadata.properties"), "w").write(_metadata(seg, extra_meta))
    open(os.path.join(d, "index_map"), "w").write("\n".join(index_map) + "\n")
    open(os.path.join(d, "columns.psf"), "wb").write(bytes(blob))


def write_star_trees(path, trees):
    """StarTreeIndexCombiner's layout beside a V3 segment (pinot-segment-local/.../startree/v2/builder/
    StarTreeIndexCombiner.java, StarTreeIndexMapUtils): every tree's buffers back to back in v3/star_tree_index (no
    magic), v3/star_tree_index_map keys "<i>.<column>.<STAR_TREE | FORWARD_INDEX>.<OFFSET | SIZE>" (column "null" for
    the tree), and the trees' metadata appended to v3/metadata.properties (repeated keys are lists, as the reference's
    own fixture writes split.order and function.column.pairs)."""
    d = os.path.join(path, "v3")
    blob, imap, meta, off = bytearray(), [], [f"startree.v2.count = {len(trees)}"], 0
    for i, st in enumerate(trees):
        parts = [("null", "STAR_TREE", st.tree)] + [(c, "FORWARD_INDEX", st.dim_fwd[c]) for c in st.dimensions] + \
                [(m, "FORWARD_INDEX", st.metric_fwd[m]) for m in st.pairs]
        for col, kind, payload in parts:
            b = np.ascontiguousarray(payload, np.uint8).tobytes()
            imap += [f"{i}.{col}.{kind}.OFFSET = {off}", f"{i}.{col}.{kind}.SIZE = {len(b)}"]
            blob += b
            off += len(b)
        meta.append(f"startree.v2.{i}.total.docs = {st.num_docs}")
        meta += [f"startree.v2.{i}.split.order = {x}" for x in st.dimensions]
        meta += [f"startree.v2.{i}.function.column.pairs = {x}" for x in st.pairs]
        meta.append(f"startree.v2.{i}.max.leaf.records = {st.max_leaf_records}")
    open(os.path.join(d, "star_tree_index"), "wb").write(bytes(blob))
    open(os.path.join(d, "star_tree_index_map"), "w").write("\n".join(imap) + "\n")
    with open(os.path.join(d, "metadata.properties"), "a") as f:
        f.write("\n".join(meta) + "\n")


def write_v1(seg, path):
    os.makedirs(path, exist_ok=True)
    open(os.path.join(path, "metadata.properties"), "w").write(_metadata(seg))
    for c, cb in seg.columns.items():
        ext = {"dictionary": ".dict", "forward_index": ".sv.raw.fwd" if cb.raw else
               (".sv.sorted.fwd" if cb.is_sorted else ".sv.unsorted.fwd"),
               "inverted_index": ".bitmap.inv", "range_index": ".bitmap.range"}
        for idx, payload in _buffers(cb):
            open(os.path.join(path, c + ext[idx]), "wb").write(payload)


def _props(path):
    kv = {}
    for line in open(path, encoding="utf-8"):
        t = line.strip()
        if not t or t[0] in "#!" or "=" not in t:
            continue
        k, v = t.split("=", 1)
        kv[k.strip().replace("\\:", ":").replace("\\=", "=")] = v.strip()
    return kv


def read_dir(path):
    """Oracle segment of a V3 or V1 segment directory (single-value dictionary columns)."""
    v3 = os.path.isdir(os.path.join(path, "v3"))
    d = os.path.join(path, "v3") if v3 else path
    meta = _props(os.path.join(d, "metadata.properties"))
    n = int(meta["segment.total.docs"])
    cols = sorted(k[len("column."):-len(".cardinality")] for k in meta if k.startswith("column.")
                  and k.endswith(".cardinality"))
    if v3:
        imap = _props(os.path.join(d, "index_map"))
        psf = open(os.path.join(d, "columns.psf"), "rb").read()

        def buf(c, idx):
            s, z = int(imap[f"{c}.{idx}.startOffset"]), int(imap[f"{c}.{idx}.size"])
            assert psf[s:s + 8] == MAGIC
            return psf[s + 8:s + z]
    out = {}
    for c in cols:
        g = lambda k: meta[f"column.{c}.{k}"]  # noqa: E731
        dt, card, bits = g("dataType"), int(g("cardinality")), int(g("bitsPerElement"))
        srt = g("isSorted") == "true"
        if meta.get(f"column.{c}.hasDictionary") == "false":  # raw: values -> sorted distinct dictionary + ids
            fwd = buf(c, "forward_index") if v3 else open(os.path.join(d, c + ".sv.raw.fwd"), "rb").read()
            values, ids = np.unique(RC.read_raw(fwd, dt, n), return_inverse=True)
            b = O.num_bits_per_value(len(values) - 1) if len(values) > 1 else 1
            out[c] = dict(dictionary=values, fwd=O.fixed_bit_pack(ids.astype(np.int32), b), bits=b, data_type=dt,
                          num_docs=n)
            continue
        if v3:
            dic, fwd = buf(c, "dictionary"), buf(c, "forward_index")
        else:
            dic = open(os.path.join(d, c + ".dict"), "rb").read()
            fwd = open(os.path.join(d, c + (".sv.sorted.fwd" if srt else ".sv.unsorted.fwd")), "rb").read()
        if dt == "STRING":
            w = int(g("lengthOfEachEntry"))
            values = np.array([dic[i * w:(i + 1) * w].split(b"\0", 1)[0].decode() for i in range(card)])
        else:
            values = np.frombuffer(dic, _NP[dt], count=card).astype(_NP[dt][1:])
        if srt:  # (start, end) doc pairs per dictId -> the dictIds they imply, packed like an unsorted column
            r = np.frombuffer(fwd, ">i4", count=2 * card).reshape(card, 2)
            ids = np.repeat(np.arange(card, dtype=np.int32), np.maximum(r[:, 1] - r[:, 0] + 1, 0))
            fwd = O.fixed_bit_pack(ids, bits).tobytes()
        out[c] = dict(dictionary=values, fwd=np.frombuffer(fwd, np.uint8), bits=bits, data_type=dt, num_docs=n)
    seg = O.segment_from_dict_ids(meta.get("segment.name", path), out)
    for c in cols:  # exact (version 2) range indexes: RangeIndexBasedFilterOperator leaves
        if v3:
            hdr = buf(c, "range_index")[:4] if f"{c}.range_index.startOffset" in imap else b""
        else:
            rp = os.path.join(d, c + ".bitmap.range")
            hdr = open(rp, "rb").read(4) if os.path.exists(rp) else b""
        seg.columns[c].has_range_index = hdr == b"\x00\x00\x00\x02"
    return seg, meta
