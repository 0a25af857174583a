// datatable.cpp -- server -> broker DataTable V4 straight from a ph_result.
//
// What the reference's server sends for the path's results (InstanceResponseBlock.toDataTable):
//   GroupByResultsBlock.getDataTable (GroupByResultsBlock.java:170-265) / AggregationResultsBlock.getDataTable
//   (AggregationResultsBlock.java:100-150), built by DataTableBuilderV4 / BaseDataTableBuilder and serialised by
//   DataTableImplV4.toBytes (DataTableImplV4.java, writeLeadingSections / serializeMetadata), all big-endian
//   (DataOutputStream):
//     int version (4), numRows, numColumns, then (start, length) of the exceptions, string dictionary, data schema,
//     fixed-size data and variable-size data sections, the sections, then int metadata length + metadata.
//   Data schema (DataSchema.toBytes): numColumns, UTF-8 names, UTF-8 ColumnDataType names.  Columns: the group-by
//   identifiers (GroupByOperator.java:76-81; stored types INT / LONG / FLOAT / DOUBLE / STRING) then one column per
//   aggregation named AggregationFunction.getResultColumnName() (`count(*)`, `sum(m)`, `sum(times(a,b))`) with its
//   intermediate type (COUNT LONG, SUM / MIN / MAX DOUBLE, DISTINCTCOUNTHLL OBJECT).
//   Fixed-size rows (DataTableUtils.computeColumnOffsets): INT / FLOAT / STRING (a string-dictionary id, assigned in
//   first-seen order, DataTableBuilderV4.setColumn(String)) 4 bytes, LONG / DOUBLE 8, OBJECT 8 = (offset into the
//   variable section, byte length); the variable section holds int objectType (ObjectSerDeUtils.ObjectType
//   HyperLogLog = 6) + HyperLogLog.getBytes() (int log2m, int byte size, RegisterSet words).
//   Metadata (BaseResultsBlock.getResultsMetadata :190-202, GroupByResultsBlock :267-275, plus caller entries):
//   int count, then per entry int MetadataKey id + (INT: 4 bytes, LONG: 8 bytes, STRING: int length + UTF-8), in
//   java.util.HashMap iteration order (emulated below: bucket index of the spread String.hashCode in the final
//   table size, insertion order within a bucket) -- so the bytes equal the reference's for the same map.
// Row order is the result's (keys ascending); the reference's server emits its IndexedTable's iteration order,
// which carries no meaning for the broker (GroupByDataTableReducer merges by key).
#include <cstring>
#include <string>
#include <unordered_map>

#include "ph_internal.h"

namespace ph {

namespace {

struct Out {
  std::vector<uint8_t> b;
  void i32(int32_t v) {
    for (int s = 24; s >= 0; s -= 8) b.push_back((uint8_t)((uint32_t)v >> s));
  }
  void i64(int64_t v) {
    for (int s = 56; s >= 0; s -= 8) b.push_back((uint8_t)((uint64_t)v >> s));
  }
  void bytes(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
  void str(const std::string& s) {
    i32((int32_t)s.size());
    bytes(s.data(), s.size());
  }
};

inline void put_be(uint8_t* p, uint64_t v, int w) {
  for (int k = 0; k < w; ++k) p[k] = (uint8_t)(v >> (8 * (w - 1 - k)));
}

// MetadataKey (DataTable.java:103-137): id and value type (0 INT, 1 LONG, 2 STRING)
struct MetaKey {
  int id;
  int type;
};
const std::unordered_map<std::string, MetaKey>& metadata_keys() {
  static const std::unordered_map<std::string, MetaKey> m = {
      {"table", {1, 2}}, {"numDocsScanned", {2, 1}}, {"numEntriesScannedInFilter", {3, 1}},
      {"numEntriesScannedPostFilter", {4, 1}}, {"numSegmentsQueried", {5, 0}}, {"numSegmentsProcessed", {6, 0}},
      {"numSegmentsMatched", {7, 0}}, {"numConsumingSegmentsQueried", {8, 0}},
      {"minConsumingFreshnessTimeMs", {9, 1}}, {"totalDocs", {10, 1}}, {"numGroupsLimitReached", {11, 2}},
      {"timeUsedMs", {12, 1}}, {"traceInfo", {13, 2}}, {"requestId", {14, 1}}, {"numResizes", {15, 0}},
      {"resizeTimeMs", {16, 1}}, {"threadCpuTimeNs", {17, 1}}, {"systemActivitiesCpuTimeNs", {18, 1}},
      {"responseSerializationCpuTimeNs", {19, 1}}, {"numSegmentsPrunedByServer", {20, 0}},
      {"numSegmentsPrunedByInvalid", {21, 0}}, {"numSegmentsPrunedByLimit", {22, 0}},
      {"numSegmentsPrunedByValue", {23, 0}}, {"explainPlanNumEmptyFilterSegments", {24, 0}},
      {"explainPlanNumMatchAllFilterSegments", {25, 0}}, {"numConsumingSegmentsProcessed", {26, 0}},
      {"numConsumingSegmentsMatched", {27, 0}}, {"numBlocks", {28, 0}}, {"numRows", {29, 0}},
      {"operatorExecutionTimeMs", {30, 1}}, {"operatorId", {31, 2}}, {"operatorExecStartTimeMs", {32, 1}},
      {"operatorExecEndTimeMs", {33, 1}}};
  return m;
}

// java.lang.String.hashCode over UTF-16 code units (the keys are ASCII) and HashMap.hash's spread
int32_t java_hash(const std::string& s) {
  uint32_t h = 0;
  for (unsigned char c : s) h = 31u * h + c;
  return (int32_t)(h ^ (h >> 16));
}

// java.util.HashMap<String, String> insertion -> iteration order
std::vector<std::pair<std::string, std::string>> hashmap_order(const std::vector<std::pair<std::string, std::string>>& ins) {
  std::vector<std::pair<std::string, std::string>> e;
  for (auto& kv : ins) {  // put(): an existing key keeps its position, takes the new value
    bool found = false;
    for (auto& x : e)
      if (x.first == kv.first) {
        x.second = kv.second;
        found = true;
      }
    if (!found) e.push_back(kv);
  }
  size_t cap = 16;
  while (e.size() > cap * 3 / 4) cap *= 2;  // resize once size exceeds the 0.75 threshold
  std::vector<std::pair<std::string, std::string>> out;
  for (size_t bucket = 0; bucket < cap; ++bucket)
    for (auto& x : e)
      if (((uint32_t)java_hash(x.first) & (cap - 1)) == bucket) out.push_back(x);
  return out;
}

std::string agg_column_name(const ph_aggregation& a) {
  static const char* fn[] = {"count", "sum", "min", "max", "distinctcounthll"};
  if (a.type == PH_AGG_COUNT) return "count(*)";
  if (a.type < 0 || a.type > PH_AGG_DISTINCTCOUNTHLL) fail(PH_ERR_INVALID_ARGUMENT, "unknown aggregation");
  std::string arg = a.column ? a.column : "";
  if (a.expr_op != PH_EXPR_NONE) {  // FunctionContext.toString of the compiled arithmetic (TransformFunctionType)
    static const char* op[] = {"", "times", "minus", "plus"};
    arg = std::string(op[a.expr_op]) + "(" + arg + "," + (a.column2 ? a.column2 : "") + ")";
  }
  return std::string(fn[a.type]) + "(" + arg + ")";
}

const char* column_type_name(int32_t t) {
  switch (t) {
    case PH_INT: return "INT";
    case PH_LONG: return "LONG";
    case PH_FLOAT: return "FLOAT";
    case PH_DOUBLE: return "DOUBLE";
    case PH_STRING: return "STRING";
    default: fail(PH_ERR_INVALID_ARGUMENT, "unknown key type");
  }
}

}  // namespace

std::vector<uint8_t> result_to_datatable(const ph_result* r, const ph_query* q, const ph_metadata_entry* extra,
                                         int32_t num_extra) {
  if (!r || !q) fail(PH_ERR_INVALID_ARGUMENT, "null result or query");
  const int nk = (int)r->keys.size(), na = (int)r->aggs.size();
  if (nk != q->num_group_by || na != q->num_aggregations)
    fail(PH_ERR_INVALID_ARGUMENT, "query does not describe this result");
  const int ncol = nk + na;
  const int64_t nrows = r->num_groups;
  // schema + fixed row layout
  std::vector<std::string> names, types;
  std::vector<int> width(ncol), off(ncol);
  int row = 0;
  for (int i = 0; i < nk; ++i) {
    names.push_back(q->group_by[i]);
    types.push_back(column_type_name(r->key_types[i]));
    width[i] = (r->key_types[i] == PH_LONG || r->key_types[i] == PH_DOUBLE) ? 8 : 4;
  }
  for (int k = 0; k < na; ++k) {
    names.push_back(agg_column_name(q->aggregations[k]));
    const int t = r->agg_types[k];
    types.push_back(t == PH_AGG_COUNT ? "LONG" : (t == PH_AGG_DISTINCTCOUNTHLL ? "OBJECT" : "DOUBLE"));
    width[nk + k] = 8;
  }
  for (int c = 0; c < ncol; ++c) {
    off[c] = row;
    row += width[c];
  }
  std::vector<uint8_t> fixed((size_t)nrows * row);
  Out var;
  std::vector<std::string> sdict;
  std::unordered_map<std::string, int32_t> sids;
  for (int64_t g = 0; g < nrows; ++g) {
    uint8_t* rowp = fixed.data() + (size_t)g * row;
    for (int i = 0; i < nk; ++i) {
      const uint8_t* src = r->keys[i].data() + (size_t)g * r->key_entry_size[i];
      uint64_t v = 0;
      switch (r->key_types[i]) {
        case PH_INT: case PH_FLOAT: {
          uint32_t u;
          memcpy(&u, src, 4);
          v = u;
          break;
        }
        case PH_LONG: case PH_DOUBLE:
          memcpy(&v, src, 8);
          break;
        default: {  // STRING: zero-padded entry -> string-dictionary id (first seen)
          const std::string s(reinterpret_cast<const char*>(src), strnlen(reinterpret_cast<const char*>(src),
                                                                          r->key_entry_size[i]));
          auto it = sids.find(s);
          if (it == sids.end()) {
            it = sids.emplace(s, (int32_t)sdict.size()).first;
            sdict.push_back(s);
          }
          v = (uint32_t)it->second;
        }
      }
      put_be(rowp + off[i], v, width[i]);
    }
    for (int k = 0; k < na; ++k) {
      uint8_t* dst = rowp + off[nk + k];
      const uint8_t* base = r->aggs[k].data();
      const int t = r->agg_types[k];
      if (t == PH_AGG_DISTINCTCOUNTHLL) {
        const int log2m = r->agg_log2m[k];
        const int m = 1 << log2m, words = m / 6 + 1;  // RegisterSet: 6 five-bit registers per int
        const uint8_t* reg = base + (size_t)g * m;
        put_be(dst, (uint32_t)var.b.size(), 4);
        put_be(dst + 4, (uint32_t)(8 + 4 * words), 4);
        var.i32(6);  // ObjectSerDeUtils.ObjectType.HyperLogLog
        var.i32(log2m);
        var.i32(4 * words);
        std::vector<uint32_t> w(words, 0);
        for (int j = 0; j < m; ++j) w[j / 6] |= (uint32_t)(reg[j] & 0x1f) << (5 * (j % 6));
        for (uint32_t x : w) var.i32((int32_t)x);
      } else {
        uint64_t v;
        memcpy(&v, base + (size_t)g * 8, 8);  // COUNT int64, SUM / MIN / MAX double bits
        put_be(dst, v, 8);
      }
    }
  }
  // metadata: results metadata in the reference's put order, then the caller's entries
  const ph_exec_stats& s = r->stats;
  std::vector<std::pair<std::string, std::string>> meta = {
      {"totalDocs", std::to_string(s.num_total_docs)},
      {"numDocsScanned", std::to_string(s.num_docs_scanned)},
      {"numEntriesScannedInFilter", std::to_string(s.num_entries_scanned_in_filter)},
      {"numEntriesScannedPostFilter", std::to_string(s.num_entries_scanned_post_filter)},
      {"numSegmentsProcessed", std::to_string(s.num_segments_processed)},
      {"numSegmentsMatched", std::to_string(s.num_segments_matched)},
      {"numConsumingSegmentsProcessed", "0"},
      {"numConsumingSegmentsMatched", "0"}};
  if (nk > 0) {
    if (s.num_groups_limit_reached) meta.push_back({"numGroupsLimitReached", "true"});
    meta.push_back({"numResizes", "0"});  // dense device tables never resize
    meta.push_back({"resizeTimeMs", "0"});
  }
  for (int32_t i = 0; i < num_extra; ++i) {
    if (!extra[i].key || !extra[i].value) fail(PH_ERR_INVALID_ARGUMENT, "null metadata entry");
    meta.push_back({extra[i].key, extra[i].value});
  }
  Out md;
  const auto ordered = hashmap_order(meta);
  md.i32((int32_t)ordered.size());
  for (auto& kv : ordered) {
    auto it = metadata_keys().find(kv.first);
    if (it == metadata_keys().end()) continue;  // serializeMetadata skips unknown keys (the count still includes them)
    md.i32(it->second.id);
    if (it->second.type == 0) md.i32((int32_t)std::stol(kv.second));
    else if (it->second.type == 1) md.i64((int64_t)std::stoll(kv.second));
    else md.str(kv.second);
  }
  // sections
  Out exc;
  exc.i32(0);  // no exceptions
  Out dict;  // DataTableBuilderV4.build always passes a (possibly empty) string dictionary
  dict.i32((int32_t)sdict.size());
  for (auto& x : sdict) dict.str(x);
  Out schema;
  schema.i32(ncol);
  for (auto& n : names) schema.str(n);
  for (auto& t : types) schema.str(t);
  Out o;
  const int32_t header = 13 * 4;
  o.i32(4);
  o.i32((int32_t)nrows);
  o.i32(ncol);
  int32_t pos = header;
  o.i32(pos);
  o.i32((int32_t)exc.b.size());
  pos += (int32_t)exc.b.size();
  o.i32(pos);
  o.i32((int32_t)dict.b.size());
  pos += (int32_t)dict.b.size();
  o.i32(pos);
  o.i32((int32_t)schema.b.size());
  pos += (int32_t)schema.b.size();
  o.i32(pos);
  o.i32((int32_t)fixed.size());
  pos += (int32_t)fixed.size();
  o.i32(pos);
  o.i32((int32_t)var.b.size());
  o.bytes(exc.b.data(), exc.b.size());
  o.bytes(dict.b.data(), dict.b.size());
  o.bytes(schema.b.data(), schema.b.size());
  o.bytes(fixed.data(), fixed.size());
  o.bytes(var.b.data(), var.b.size());
  o.i32((int32_t)md.b.size());
  o.bytes(md.b.data(), md.b.size());
  return std::move(o.b);
}

}  // namespace ph
