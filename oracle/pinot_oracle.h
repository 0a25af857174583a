/*
 * pinot_oracle.h -- CPU restatement of Apache Pinot's server-side per-segment
 * filter -> aggregation / group-by path (reference: weixiangsun/pinot @ 1.1.0-SNAPSHOT).
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker ("oracle") and the
 * timed CPU baseline ("cpu_baseline.kind = port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product (libpinot_hip.so) never links
 * or calls anything here.
 *
 * Parity pinning: the restatement is checked against the reference's own known-answer
 * tests over pinot-core/src/test/resources/data/test_data-sv.avro
 * (InterSegmentAggregationSingleValueQueriesTest.java:45-283,
 *  InterSegmentGroupBySingleValueQueriesTest.java:62-140) and the closed-form
 * FastFilteredCountTest / RangeQueriesTest data (see tests/test_oracle_kat.py).
 */
#ifndef PINOT_ORACLE_H
#define PINOT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* PinotDataBitSet.getNumBitsPerValue (pinot-segment-local/.../io/util/PinotDataBitSet.java:59-70) */
int or_num_bits_per_value(int32_t max_value);
/* FixedBitSVForwardIndexWriter length: ((long)N*b+7)/8 (FixedBitSVForwardIndexWriter.java:42) */
int64_t or_fixed_bit_num_bytes(int64_t num_values, int bits);
/* PinotDataBitSet.writeInt loop over all values (PinotDataBitSet.java:138-165); buffer must be zeroed */
void or_fixed_bit_write(const int32_t* values, int64_t n, int bits, uint8_t* out);
/* PinotDataBitSet.readInt (PinotDataBitSet.java:78-100) */
int32_t or_fixed_bit_read(const uint8_t* buf, int64_t index, int bits);
/* PinotDataBitSet.readInt(startIndex, numBits, length, buffer) (PinotDataBitSet.java:102-136) */
void or_fixed_bit_read_range(const uint8_t* buf, int64_t start, int bits, int32_t length, int32_t* out);

/* clearspring stream 2.7.0 MurmurHash.hashLong (seed 0) and MurmurHash.hash(byte[]) (seed -1),
 * restated from the published algorithm; pinned by the DISTINCTCOUNTHLL KATs. */
int32_t or_murmur_hash_long(int64_t v);
int32_t or_murmur_hash_bytes(const uint8_t* data, int32_t len, int32_t seed);
/* HyperLogLog.offerHashed register update for log2m (clearspring HyperLogLog.offerHashed(int)) */
void or_hll_offer_hashed(uint8_t* registers, int log2m, int32_t hash);
/* HyperLogLog.cardinality() */
int64_t or_hll_cardinality(const uint8_t* registers, int log2m);

/* ---- segment / query model (dictId space; literals are mapped by oracle.py) ---- */
typedef struct {
  int32_t cardinality;
  int32_t bits;               /* bitsPerElement (unsorted) */
  const uint8_t* fwd;         /* fixed-bit big-endian forward index, NULL when sorted */
  const int32_t* sorted;      /* [card][2] (start,end inclusive) when the column is sorted */
  const double* values;       /* dictId -> value as double (numeric), NULL for STRING */
  const int64_t* hash_longs;  /* dictId -> long passed to MurmurHash.hashLong (INT/LONG) or NULL */
  const int32_t* hash_ints;   /* dictId -> precomputed 32-bit hash (STRING/FLOAT/DOUBLE) or NULL */
  const int32_t* global_ids;  /* dictId -> id in the table-level sorted value union (group keys) */
} or_column;

typedef struct {
  int32_t num_docs;
  int32_t num_columns;
  const or_column* columns;
} or_segment;

enum { OR_F_LEAF = 0, OR_F_AND = 1, OR_F_OR = 2, OR_F_NOT = 3, OR_F_ALL = 4, OR_F_NONE = 5 };
typedef struct {
  int32_t op;                 /* OR_F_* */
  int32_t arg;                /* LEAF: column index ; AND/OR: number of children */
  const uint8_t* match;       /* LEAF: per-dictId 0/1 */
  int32_t is_scan;            /* LEAF: counted in numEntriesScannedInFilter; AND: nidx << 8 | nscan when its children
                                 are nidx index-based ones then nscan scans (applyAnd statistic), else 0 */
} or_filter_op;               /* postfix program */

enum { OR_AGG_COUNT = 0, OR_AGG_SUM = 1, OR_AGG_MIN = 2, OR_AGG_MAX = 3, OR_AGG_HLL = 4 };
typedef struct {
  int32_t num_filter_ops;     /* 0 = no filter */
  const or_filter_op* filter;
  int32_t num_group_by;
  const int32_t* group_cols;
  const int64_t* group_global_card;   /* per group column: size of the value union */
  int32_t num_aggs;
  const int32_t* agg_fn;
  const int32_t* agg_col;     /* -1 for COUNT(*) */
  int32_t log2m;
  int64_t num_groups_limit;   /* per segment (InstancePlanMakerImplV2 numGroupsLimit) */
  /* 2-operand expression arguments (TransformOperator, ProjectPlanNode.java:82): agg_op[k] = 0 plain column,
   * 1 mult, 2 sub, 3 add over agg_col[k] and agg_col2[k], evaluated per row in double
   * (MultiplicationTransformFunction.java:89-104, SubtractionTransformFunction.java:99-124); NULL = none */
  const int32_t* agg_col2;
  const int32_t* agg_op;
} or_query;

typedef struct {
  int64_t num_groups;
  uint64_t* keys;             /* [num_groups] mixed-radix key over global ids, column 0 least significant */
  double* aggs;               /* [num_groups][num_aggs] (HLL slots unused) */
  uint8_t* hll;               /* [num_groups][num_hll][2^log2m] */
  int32_t num_hll;
  int64_t num_docs_scanned;
  int64_t num_entries_scanned_in_filter;
  int64_t num_entries_scanned_post_filter;
  int64_t num_total_docs;
  int32_t num_groups_limit_reached;
} or_result;

/* ServerQueryExecutorV1Impl -> GroupByCombineOperator / AggregationCombineOperator restated:
 * one task per segment on a pool of num_threads workers, merged into a shared table. */
int or_execute(const or_query* q, const or_segment* segs, int32_t num_segs, int32_t num_threads,
               or_result* out);
void or_result_free(or_result* r);

#ifdef __cplusplus
}
#endif
#endif
