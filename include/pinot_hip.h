/*
 * pinot_hip.h -- C-ABI of libpinot_hip.so, the MI355X-native server-side segment execution path
 * (filter -> aggregation / group-by on immutable, dictionary-encoded segments pinned in HBM).
 *
 * Plain C: POD structs, pointers and sizes, int status codes, no C++ or torch types.  Every entry
 * point is thread-safe.  The Java binding (JNI for JDK 11/17/20, FFM for JDK >= 22) and the Python
 * ctypes binding both bind exactly these symbols.
 *
 * Reference interfaces each entry point replaces (weixiangsun/pinot @ 1.1.0-SNAPSHOT):
 *   ph_segment_pin / ph_segment_unpin
 *       ImmutableSegmentLoader.load (pinot-segment-local/.../indexsegment/immutable/
 *       ImmutableSegmentLoader.java:67-149) and ImmutableSegmentImpl.destroy (:249), hooked from
 *       BaseTableDataManager.addSegment (pinot-core/.../data/manager/BaseTableDataManager.java:232).
 *       The column buffers are the PinotDataBuffer slices of columns.psf
 *       (SingleFileIndexDirectory.java:279-305): fixed-bit forward index, sorted index, dictionary,
 *       bitmap inverted index, all big-endian exactly as on disk.
 *   ph_query_execute
 *       PlanMaker.makeInstancePlan(...).execute() (pinot-core/.../plan/maker/PlanMaker.java:37-67,
 *       ServerQueryExecutorV1Impl.java:369-376) for the filter -> aggregation / group-by shapes:
 *       FilterPlanNode.run (:83-114), AggregationPlanNode.run (:75), GroupByPlanNode.run (:57),
 *       GroupByCombineOperator.mergeResults (:223-252).
 *   ph_filter_execute
 *       FilterPlanNode.run (pinot-core/.../plan/FilterPlanNode.java:83-114) -> a BaseFilterOperator
 *       (BaseFilterOperator.java:59-92: getTrues / canOptimizeCount / getNumMatchingDocs), the segment-level plug
 *       point (PlanMaker.makeSegmentPlanNode, PlanMaker.java:53; FilterOperatorUtils.setImplementation :40).
 *   ph_result_*
 *       GroupByResultsBlock / AggregationResultsBlock contents (GroupByResultsBlock.java:62,86;
 *       AggregationResultsBlock.java:50) and ExecutionStatistics (GroupByOperator.java:143-148).
 *   ph_result_datatable
 *       DataTableImplV4.toBytes of GroupByResultsBlock.getDataTable / AggregationResultsBlock.getDataTable
 *       (pinot-common/.../datatable/DataTableImplV4.java, GroupByResultsBlock.java:170).
 *   ph_raw_forward_index_read (+ ph_column_desc.raw_forward_index)
 *       FixedByteChunkSVForwardIndexReader / BaseChunkForwardIndexReader (pinot-segment-local/.../readers/
 *       forward/BaseChunkForwardIndexReader.java:57-105) behind ForwardIndexReaderFactory.createRawIndexReader.
 *   ph_fixed_bit_pack
 *       FixedBitSVForwardIndexWriter.putDictId (pinot-segment-local/.../io/writer/impl/
 *       FixedBitSVForwardIndexWriter.java:39-50) -- the on-disk forward-index format.
 *   ph_last_error
 *       the message of the Java exception the caller raises (BadQueryRequestException for
 *       PH_ERR_BAD_QUERY, PredicateEvaluatorProvider.java:92-95; RuntimeException otherwise, which
 *       GroupByCombineOperator turns into an ExceptionResultsBlock, :236-239).
 */
#ifndef PINOT_HIP_H
#define PINOT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status codes */
#define PH_OK 0
#define PH_ERR_INVALID_ARGUMENT 1 /* caller bug (null pointer, bad size) */
#define PH_ERR_BAD_QUERY 2        /* BadQueryRequestException: unknown column, unparsable literal */
#define PH_ERR_UNSUPPORTED 3      /* shape not on the GPU path: caller falls back to the CPU plan */
#define PH_ERR_DEVICE 4           /* HIP runtime / kernel error */
#define PH_ERR_OUT_OF_MEMORY 5    /* HBM budget exhausted */
#define PH_ERR_CANCELLED 6        /* ph_query.interrupt set or ph_query.end_time_ms passed: the caller raises the
                                     reference's timeout / cancellation (QueryException EXECUTION_TIMEOUT,
                                     QUERY_CANCELLATION; BaseOperator.java:39, GroupByCombineOperator.java:225-234) */

/* ------------------------------------------------------------------ handles */
typedef struct ph_ctx ph_ctx;         /* one per GPU; owns streams, scratch, pinned-segment registry */
typedef struct ph_segment ph_segment; /* an immutable segment resident in HBM */
typedef struct ph_result ph_result;   /* host-side result of one query */

/* Stored data types of dictionary-encoded single-value columns (FieldSpec.DataType). */
typedef enum { PH_INT = 0, PH_LONG = 1, PH_FLOAT = 2, PH_DOUBLE = 3, PH_STRING = 4 } ph_data_type;

/* ------------------------------------------------------------------ segment description */
typedef struct {
  const char* name;
  int32_t data_type;            /* ph_data_type */
  int32_t cardinality;          /* column.<c>.cardinality */
  int32_t bits_per_element;     /* column.<c>.bitsPerElement = getNumBitsPerValue(card - 1) */
  int32_t is_sorted;            /* column.<c>.isSorted */
  /* forward_index: unsorted -> fixed-bit packed dictIds, MSB-first, big-endian, ((N*b+7)/8) bytes
   *                sorted   -> int32 BE (startDocId, endDocId) pairs, 2*card entries
   *                (SortedIndexReaderImpl.java:37-42) */
  const void* forward_index;
  uint64_t forward_index_size;
  /* dictionary: sorted ascending, fixed width BE (INT 4, LONG 8, FLOAT 4, DOUBLE 8); STRING: UTF-8
   * zero-padded to dictionary_entry_size (SegmentDictionaryCreator.java:100-276) */
  const void* dictionary;
  uint64_t dictionary_size;
  int32_t dictionary_entry_size;
  /* optional bitmap inverted index: uint32 BE offsets[card+1] then portable RoaringBitmap blobs
   * (BitmapInvertedIndexWriter.java:33-96); NULL when the column has none */
  const void* inverted_index;
  uint64_t inverted_index_size;
  /* 1: forward_index is a raw (no-dictionary) single-value chunk forward index of a fixed-width stored type
   * (FixedByteChunkSVForwardIndexReader / FixedBytePower2ChunkSVForwardIndexReader format,
   * BaseChunkForwardIndexReader.java:57-105; PASS_THROUGH, LZ4, LZ4_LENGTH_PREFIXED or SNAPPY chunks), as
   * ForwardIndexReaderFactory.createRawIndexReader (:75-82) reads it; cardinality, bits_per_element and the
   * dictionary are then ignored (the pin decodes the values once and dictionary-encodes them in HBM) */
  int32_t raw_forward_index;
  /* optional range index (BitSlicedRangeIndexCreator.java:38-131: int32 BE version 2, int64 BE min, then the serialized
   * RoaringBitmap RangeBitmap; V1 file <column>.bitmap.range, V3 index_map key range_index); NULL when the column has
   * none.  A version-2 (exact) index makes RANGE, and EQ on a column without an inverted index, a
   * RangeIndexBasedFilterOperator leaf (FilterOperatorUtils.java:97-120): index-based for the AND order and the
   * statistics (no entries scanned in filter).  On a dictionary column the RangeBitmap is parsed at pin and such a
   * leaf's doc bitmap is composed from its bit slices on the device (BitSlicedRangeIndexReader.getMatchingDocIds
   * :123-211); on a raw column the leaf scans the dictIds the pin encoded (same doc set).  A version-1 index over
   * dictIds (RangeIndexCreator, type "INT") makes RANGE an index-based leaf whose statistic is its boundary ranges'
   * docs (RangeIndexBasedFilterOperator.evaluateLegacyRangeFilter :82-107); over raw values it is UNSUPPORTED at query
   * time.  (An array / run container wider than a bitmap container, which RoaringBitmap never writes, makes the
   * exact leaf scan the dictIds instead.) */
  const void* range_index;
  uint64_t range_index_size;
  /* > 0: build the column's DISTINCTCOUNTHLL table for this log2m at pin -- the per-dictId (register, rank) pairs of
   * clearspring HyperLogLog.offer(dictionary value) (DistinctCountHLLAggregationFunction.java:438-447) -- so no
   * query pays for it; 0: the first query that needs it builds it */
  int32_t hll_log2m;
} ph_column_desc;

typedef struct {
  const char* name;             /* segment.name */
  int32_t num_docs;             /* segment.total.docs */
  int32_t num_columns;
  const ph_column_desc* columns;
} ph_segment_desc;

/* ------------------------------------------------------------------ query description */
typedef enum { PH_PRED_EQ = 0, PH_PRED_NOT_EQ = 1, PH_PRED_IN = 2, PH_PRED_NOT_IN = 3, PH_PRED_RANGE = 4 }
    ph_predicate_type;

typedef struct {
  int32_t type;                 /* ph_predicate_type */
  const char* column;
  int32_t num_values;           /* EQ / NOT_EQ: 1; IN / NOT_IN: n */
  const char* const* values;    /* literals as strings, as Pinot's Predicate keeps them */
  const char* lower;            /* RANGE bounds; "*" = RangePredicate.UNBOUNDED */
  const char* upper;
  int32_t lower_inclusive;
  int32_t upper_inclusive;
} ph_predicate;

typedef enum { PH_FILTER_AND = 0, PH_FILTER_OR = 1, PH_FILTER_NOT = 2, PH_FILTER_PREDICATE = 3 } ph_filter_type;

typedef struct {
  int32_t type;                 /* ph_filter_type (FilterContext.Type) */
  int32_t num_children;
  const int32_t* children;      /* indices into ph_query.filter_nodes */
  int32_t predicate;            /* PREDICATE: index into ph_query.predicates */
} ph_filter_node;

typedef enum { PH_AGG_COUNT = 0, PH_AGG_SUM = 1, PH_AGG_MIN = 2, PH_AGG_MAX = 3, PH_AGG_DISTINCTCOUNTHLL = 4 }
    ph_aggregation_type;

/* 2-operand expression argument of SUM / MIN / MAX: `column <op> column2`, evaluated per row like the reference's
 * TransformOperator (ProjectPlanNode.java:82, AggregationFunctionUtils.java:86): MultiplicationTransformFunction
 * ("mult"), SubtractionTransformFunction ("sub"), AdditionTransformFunction ("add"), DOUBLE results.  Integer
 * operands whose results fit int64 are computed exactly in int64 (== the double result while |value| < 2^53). */
typedef enum { PH_EXPR_NONE = 0, PH_EXPR_MULT = 1, PH_EXPR_SUB = 2, PH_EXPR_ADD = 3 } ph_expr_op;

typedef struct {
  int32_t type;                 /* ph_aggregation_type */
  const char* column;           /* NULL for COUNT(*); first operand of an expression */
  int32_t log2m;                /* DISTINCTCOUNTHLL; 0 = default 8 (CommonConstants.java:96-97) */
  const char* column2;          /* second operand (expr_op != PH_EXPR_NONE), else NULL */
  int32_t expr_op;              /* ph_expr_op */
} ph_aggregation;

typedef struct {
  int32_t num_filter_nodes;
  const ph_filter_node* filter_nodes;
  int32_t filter_root;          /* -1: no WHERE clause */
  int32_t num_predicates;
  const ph_predicate* predicates;
  int32_t num_group_by;
  const char* const* group_by;  /* identifiers (DictionaryBasedGroupKeyGenerator columns) */
  int32_t num_aggregations;
  const ph_aggregation* aggregations;
  int64_t num_groups_limit;     /* per-segment numGroupsLimit (InstancePlanMakerImplV2.java:72-73) */
  /* Interruption (BaseOperator.nextBlock checks Tracing.ThreadAccountantOps.isInterrupted, BaseOperator.java:39;
   * the combine waits until QueryContext.getEndTimeMs, GroupByCombineOperator.java:225-234).  A call checks both
   * before its launches and between scan batches (with either set, a scan is cut into batches of ~128M docs and
   * the stream is drained between them), and returns PH_ERR_CANCELLED. */
  int64_t end_time_ms;                /* wall-clock deadline, ms since the Unix epoch; 0 = none */
  const volatile int32_t* interrupt;  /* the caller sets *interrupt != 0 to cancel; NULL = none */
  /* Segment group trim (GroupByOperator.java:114-130): with a group-by, ORDER BY and min_segment_group_trim_size > 0
   * (query option minSegmentGroupTrimSize; <= 0 = off, the default -1), every segment holding more groups than
   * GroupByUtils.getTableCapacity(limit, min_segment_group_trim_size) = max(5 * limit, min) keeps only that many,
   * chosen by TableResizer.trimInSegmentResults (a heap over the ORDER BY values, fed in the group-key iterator's
   * order), before the combine merges the segments.  DISTINCTCOUNTHLL in the ORDER BY is PH_ERR_UNSUPPORTED. */
  int32_t num_order_by;
  const struct ph_order_by* order_by;
  int32_t limit;                      /* the query's LIMIT */
  int32_t min_segment_group_trim_size;
  /* query option skipStarTree (QueryContext.isSkipStarTree): 1 = never answer from a segment's star-tree */
  int32_t skip_star_tree;
} ph_query;

/* one ORDER BY expression: a group-by column (index into group_by) or an aggregation (index into aggregations) */
typedef enum { PH_ORDER_GROUP_BY = 0, PH_ORDER_AGGREGATION = 1 } ph_order_kind;
typedef struct ph_order_by {
  int32_t kind;                 /* ph_order_kind */
  int32_t index;
  int32_t asc;                  /* 1 ASC, 0 DESC */
} ph_order_by;

typedef struct {
  int64_t num_docs_scanned;                /* matched docs */
  int64_t num_entries_scanned_in_filter;   /* the docs the reference's scan iterators examine */
  int64_t num_entries_scanned_post_filter; /* numDocsScanned x projected columns */
  int64_t num_total_docs;
  int64_t num_segments_processed;
  int64_t num_segments_matched;
  int32_t num_groups_limit_reached;
  int32_t sum_precision_flag;              /* 1 if an integer SUM reached 2^53 (double rounding differs) */
  double device_ms;                        /* kernel time of the query, HIP events */
  double host_ms;                          /* planning + result materialisation */
  int32_t plan_mode;                       /* physical plan: -2 index-only count (FastFilteredCount), -1
                                              metadata, 0 count, 1 aggregation, 2 LDS group table, 3 HBM
                                              atomic group table, 4 partitioned, 5 HBM hash group table */
  int32_t limit_pass;                      /* numGroupsLimit emulation: 0 no segment could reach the limit, 1 the
                                              untruncated scan's table held < limit keys (no pass needed), 2 the
                                              first-seen pass and the truncating scan ran */
  int32_t scan_kernel;                     /* the scan's kernel (PH_KERNEL_*): which hand-written form ran */
  int32_t num_devices;                     /* devices whose segments the query scanned (multi-device contexts) */
  double merge_ms;                         /* multi-device: combining the devices' partial tables (RCCL / local) */
  double finalize_ms;                      /* multi-device: turning the merged key shards into the result */
  double scan_ms;                          /* multi-device: wall time of the devices' scans into their partial tables
                                              (host_ms - scan_ms - merge_ms - finalize_ms = planning + assembly) */
  int64_t num_segments_star_tree;          /* segments answered from a star-tree (GroupByPlanNode :77-99,
                                              AggregationPlanNode :122-141) */
} ph_exec_stats;

/* ph_exec_stats.scan_kernel */
enum {
  PH_KERNEL_NONE = 0,          /* no scan (metadata / index-only answer, or nothing to scan) */
  PH_KERNEL_SCAN = 1,          /* k_scan<MODE, ...>: the generic persistent scan */
  PH_KERNEL_AGG_LEAN = 2,      /* k_agg_lean: one packed integer column, aggregation only */
  PH_KERNEL_AGG_SPARSE = 3,    /* k_agg_sparse: gathers of the docs of selective inverted-index bitmaps */
  PH_KERNEL_GROUP_LDS_LEAN = 4,/* k_group_lds_lean: LDS-private group tables */
  PH_KERNEL_PART_LEAN = 5,     /* k_part_scan + k_part_agg: partitioned group-by, one tile of loads in flight */
  PH_KERNEL_PART_LEAN2 = 6,    /* k_part_scan2 + k_part_agg: partitioned group-by, two tiles of loads in flight */
  PH_KERNEL_PART_SCAN = 7,     /* k_scan<MODE_PARTITION> + k_part_agg: partitioned group-by with gathers */
  PH_KERNEL_PART_REG = 8,      /* k_part_reg + k_part_agg: partitioned group-by, register-direct decode */
  PH_KERNEL_COUNT_REG = 9,     /* k_count_reg: COUNT(*) over RANGE / ALL / sorted leaves, register-direct decode */
  /* 10: retired (round 3's k_agg_reg, slower than k_agg_lean everywhere measured; removed in round 6) */
  PH_KERNEL_GROUP_REG = 11,    /* k_group_reg: k_group_lds_lean's group-by in the register-direct form */
  PH_KERNEL_GROUP_SPARSE = 12, /* k_group_sparse: group-by over selective inverted-index ANDs, matched-doc gathers */
  /* 13: retired (round 4's wave-private-ring kernel A, removed in round 5) */
  PH_KERNEL_AGG_CONTAINERS = 14, /* k_agg_sparse straight from the roaring containers of an EQ / IN inverted leaf
                                    (no doc bitmaps; BitmapInvertedIndexReader.java:45-62) */
  PH_KERNEL_GROUP_CONTAINERS = 15 /* k_group_sparse with each chunk's leaf bitmaps built in LDS from the roaring
                                     containers (no doc bitmaps in HBM) */
};

/* ------------------------------------------------------------------ context */
int ph_ctx_create(int32_t device_ordinal, ph_ctx** out);
/* One context over a set of GPUs of one node -- a Pinot server's JVM combines every segment of a query in-process
 * (GroupByCombineOperator.java:125-197).  ph_segment_pin places each segment on the device with the fewest pinned
 * docs; ph_query_execute scans every device's segments there (one host thread each) into dense partial tables over
 * one set of table-level dictionaries and merges them in the library: RCCL reduce-scatter over xGMI when the devices
 * are distinct (each device then finalises its key shard), a device copy + reduce kernel when `device_ordinals`
 * repeat a device (logical shards); shapes the dense tables do not serve merge per-device results by group value.
 * The result equals ph_query_execute's over one device (DOUBLE SUM within 1e-9 relative: summation order). */
int ph_ctx_create_multi(const int32_t* device_ordinals, int32_t num_devices, ph_ctx** out);
int32_t ph_ctx_num_devices(const ph_ctx* ctx);
/* How a multi-device context merges its devices' dense partial tables (a reduce-scatter by key shard, either way):
 * PH_TRANSPORT_PEER (default) -- each device gathers its key shard of the others' tables by peer copy over xGMI and
 * reduces it with a kernel; PH_TRANSPORT_RCCL -- ncclReduceScatter over xGMI, its communicators created here (not in
 * the first query).  RCCL needs distinct device ordinals; logical shards sharing a device always take PEER.
 * Replaces the cross-server half of GroupByCombineOperator's merge (GroupByCombineOperator.java:125-197). */
#define PH_TRANSPORT_PEER 0
#define PH_TRANSPORT_RCCL 1
int ph_ctx_set_multi_transport(ph_ctx* ctx, int32_t transport);
int ph_ctx_destroy(ph_ctx* ctx);
/* Plan / kernel-form overrides of a context (tests and tuning sweeps; the library reads no environment).  `name` is
 * one of the options below; PH_OPTION_UNSET restores the planner's own choice.  Presence-style options act when set
 * to any value.  PH_ERR_INVALID_ARGUMENT for an unknown name.
 *   roaring_atomic     inverted-leaf doc bitmaps by the device-atomic build (k_roaring_or) instead of per chunk
 *   agg_cont / group_cont   0/1: k_agg_sparse / k_group_sparse straight from the roaring containers (group_cont:
 *                      opt-in, measured slower on the inverted SSB flight)
 *   agg_sparse / group_sparse  0/1: force the sparse (matched-doc gather) aggregation / group-by plans off / on
 *   disable_partition, no_group_cache, limit_eager, stat_fuse (off), part_generic, agg_generic, lds_generic,
 *   count_generic, lds_lean, part_lds, part_flush_first, part_serial: presence -- force the named alternative form
 *   lds_table_max, tile_words, group_reg_lg, interrupt_chunks, part_klo, part_batch_rows, part_depth, part_sets,
 *   part_wg_per_cu, part_slices, part_mm_blind, part_ring_log2: the value
 *   multi_host_merge   presence: a multi-device context merges by group value instead of dense partials
 *   sparse_c           2/4/8: the sparse kernels' register-direct leaf loads (2: every leaf's loads of a step in
 *                      flight at once, leaves <= 8 bits only; 4 -- the default -- / 8: leaf by leaf, fewer registers) */
#define PH_OPTION_UNSET INT64_MIN
int ph_ctx_set_option(ph_ctx* ctx, const char* name, int64_t value);
/* Launch on an external HIP stream (e.g. torch's current stream); NULL restores the context's own. */
int ph_ctx_set_stream(ph_ctx* ctx, void* hip_stream);

/* ------------------------------------------------------------------ segments */
/* Copies the column buffers into HBM and derives, on the pin stream, what queries read besides them: the
 * frame-of-reference value stream of every INT / LONG column (value - min in bits(max - min), read instead of a
 * dictionary gather per row) and the requested DISTINCTCOUNTHLL tables (hll_log2m).  The caller's buffers may be
 * released when it returns. */
int ph_segment_pin(ph_ctx* ctx, const ph_segment_desc* desc, ph_segment** out);
/* Validates a segment descriptor without a device: what ph_segment_pin would refuse, and why (ph_last_error).
 * PH_ERR_INVALID_ARGUMENT for a malformed descriptor; PH_ERR_UNSUPPORTED for a segment the GPU path does not serve:
 * a packed stream (forward index, or the value stream derived from it) of 2 GiB or more, past the kernels' 32-bit
 * buffer offsets -- the plan maker then keeps the segment on the CPU plan (GpuSegmentRegistry). */
int ph_segment_check(const ph_segment_desc* desc);
/* Pin a segment straight from its on-disk directory (replaces ImmutableSegmentLoader.load's index-buffer path,
 * ImmutableSegmentLoader.java / SingleFileIndexDirectory.java:72,213-305): V3 (<dir>/v3/: metadata.properties,
 * index_map, columns.psf) or V1 (one file per index).  `columns`
 * selects the columns to pin (NULL / 0: every single-value dictionary or fixed-width raw column); a requested
 * multi-value or variable-width raw column is PH_ERR_UNSUPPORTED. */
int ph_segment_load_dir(ph_ctx* ctx, const char* segment_dir, const char* const* columns, int32_t num_columns,
                        ph_segment** out);
int ph_segment_unpin(ph_segment* seg);
/* HBM held for the segment: its pinned columns plus the per-column caches queries derived from them
 * (re-encoded value streams, HLL hash tables, dictId remaps to table-level dictionaries). */
int64_t ph_segment_device_bytes(const ph_segment* seg);
int32_t ph_segment_num_docs(const ph_segment* seg);
int32_t ph_segment_device(const ph_segment* seg);  /* index into the context's device set */

/* Star-tree index of a pinned segment (StarTreeV2: StarTreeIndexContainer / StarTreeLoaderUtils.loadStarTreeV2,
 * pinot-segment-local/.../startree/v2/store/StarTreeLoaderUtils.java): the buffers of one star-tree in
 * star_tree_index as star_tree_index_map names them.  The records are pinned beside the segment (the dimensions with
 * the segment's own dictionaries, the function-column pair columns as raw columns); a later query whose aggregations
 * are all pairs of the tree, whose filter is an AND of per-column predicates (ORs on one column) over tree dimensions
 * and whose group-by columns are tree dimensions is answered from it, as GroupByPlanNode.java:77-99 /
 * AggregationPlanNode.java:122-141 choose it: StarTreeFilterOperator's traversal on the host
 * (StarTreeFilterOperator.java:207-358) gives the star-tree documents, the remaining predicates and the
 * aggregation over the pair columns run in the same kernels as any query (COUNT sums count__*, SUM / MIN / MAX read
 * sum__ / min__ / max__).  A pair of another function (e.g. distinctCountHLL__c) is recorded: a query it would serve
 * is PH_ERR_UNSUPPORTED (CPU plan). */
typedef struct {
  const void* tree;             /* the STAR_TREE buffer (OffHeapStarTree.java:45-83 format, little-endian) */
  uint64_t tree_size;
  int32_t num_docs;             /* startree.v2.<i>.total.docs */
  int32_t num_dimensions;       /* must equal the tree's dimensions (split order) */
  const char* const* dimensions;
  const void* const* dimension_forward_index;  /* <dim>.FORWARD_INDEX: fixed-bit dictIds at the column's bit width */
  const uint64_t* dimension_forward_index_size;
  int32_t num_metrics;          /* startree.v2.<i>.function.column.pairs ("count__*", "sum__col", ...) */
  const char* const* metrics;
  const void* const* metric_forward_index;     /* <pair>.FORWARD_INDEX raw forward index (LONG count, DOUBLE others);
                                                  NULL for a pair of another function */
  const uint64_t* metric_forward_index_size;
} ph_star_tree_desc;
int ph_segment_add_star_tree(ph_segment* seg, const ph_star_tree_desc* desc);
int32_t ph_segment_num_star_trees(const ph_segment* seg);
/* Host-only parse of a STAR_TREE buffer (OffHeapStarTree's checks: magic, version, header size, node count). */
int ph_star_tree_check(const void* tree, uint64_t tree_size, int32_t* num_nodes, int32_t* num_dimensions);

/* Table-level sorted value union for a column (group keys share ids across segments and GPUs).
 * Optional: without it the union of the queried segments' dictionaries is used. */
int ph_table_set_dictionary(ph_ctx* ctx, const char* column, int32_t data_type, const void* values, int64_t count,
                            int32_t entry_size);

/* Table schema type of a column (Schema / FieldSpec.getDataType, pinot-spi Schema.java).  Value columns take
 * their type from the queried segments; a call that queries no segment holding the column (an empty rank of a
 * multi-GPU query) takes it from here, so every rank builds the same dense layout.  A dense call that needs a
 * value column's type and has neither fails with PH_ERR_INVALID_ARGUMENT. */
int ph_table_set_column_type(ph_ctx* ctx, const char* column, int32_t data_type);

/* ------------------------------------------------------------------ queries */
int ph_query_execute(ph_ctx* ctx, const ph_query* query, ph_segment* const* segments, int32_t num_segments,
                     ph_result** out);
/* Segment-level filter: the drop-in behind FilterPlanNode.run (pinot-core/.../plan/FilterPlanNode.java:83-114), for a
 * GpuFilterOperator extends BaseFilterOperator (BaseFilterOperator.java:33-112) whose getTrues() returns a
 * BitmapDocIdSet (BitmapDocIdSet.java:29) and whose canOptimizeCount() / getNumMatchingDocs() (:59-68) answer from the
 * count, so the reference's own operators above it (selection, projection, the ~80 aggregation functions, filtered
 * aggregations) run unchanged over the GPU's doc set.  `query` contributes its filter only (filter_nodes, predicates,
 * filter_root; group-by, aggregations, ordering and trim are ignored); the planning is ph_query_execute's (same leaf
 * choice, same evaluators).  doc_words: NULL for the count alone, else >= ceil(num_docs / 64) words receiving the
 * doc bitmap -- bit i of word w is doc 64 w + i, bits past num_docs zero (the long[] layout of
 * org.roaringbitmap.BitSetUtil.bitmapOf(long[]) / java.util.BitSet.valueOf).  stats (may be NULL): num_docs_scanned
 * = matching docs, num_entries_scanned_in_filter = the reference's statistic for the segment's filter operator tree
 * (BlockDocIdSet.getNumEntriesScannedInFilter), num_total_docs, device_ms, scan_kernel.  No filter (filter_root < 0)
 * is MatchAllFilterOperator: every doc, answered without a launch. */
int ph_filter_execute(ph_ctx* ctx, const ph_query* query, ph_segment* segment, uint64_t* doc_words, uint64_t num_words,
                      ph_exec_stats* stats);
int ph_result_destroy(ph_result* r);
int ph_result_stats(const ph_result* r, ph_exec_stats* out);
/* number of result rows: non-empty groups (group-by) or 1 (aggregation-only) */
int64_t ph_result_num_groups(const ph_result* r);
/* group-key values of group-by column i for every row, in row order: INT int32, LONG int64,
 * FLOAT float, DOUBLE double, STRING entry_size-byte zero-padded UTF-8 (entry_size from
 * ph_result_key_entry_size) */
int ph_result_key_entry_size(const ph_result* r, int32_t group_by_index);
/* stored ph_data_type of group-by column i's key values */
int ph_result_key_type(const ph_result* r, int32_t group_by_index);
int ph_result_group_keys(const ph_result* r, int32_t group_by_index, void* out);
/* zero-copy views of the same columns, valid until ph_result_destroy (results must be destroyed before
 * their context) */
const void* ph_result_key_data(const ph_result* r, int32_t group_by_index);
/* intermediate result of aggregation i for every row: COUNT int64, SUM/MIN/MAX double,
 * DISTINCTCOUNTHLL uint8[2^log2m] raw registers (HyperLogLog.addAll = register-wise max) */
int ph_result_aggregation(const ph_result* r, int32_t aggregation_index, void* out);
const void* ph_result_aggregation_data(const ph_result* r, int32_t aggregation_index);

/* ------------------------------------------------------------------ server -> broker DataTable */
/* The result as the DataTable V4 bytes the reference's server returns for it (InstanceResponseBlock.toDataTable:
 * GroupByResultsBlock.getDataTable :170 / AggregationResultsBlock.getDataTable, DataTableBuilderV4,
 * DataTableImplV4.toBytes): group-by identifiers + one intermediate-result column per aggregation, results metadata
 * (BaseResultsBlock.getResultsMetadata) followed by the caller's `extra` entries (e.g. numSegmentsQueried,
 * timeUsedMs, requestId; MetadataKey names, DataTable.java:103-137), in java.util.HashMap order.  `q` is the query
 * the result came from (column names).  out == NULL: only *size is set; otherwise capacity must be >= *size. */
typedef struct {
  const char* key;
  const char* value;
} ph_metadata_entry;
int ph_result_datatable(const ph_result* r, const ph_query* q, const ph_metadata_entry* extra, int32_t num_extra,
                        void* out, uint64_t capacity, uint64_t* size);

/* ------------------------------------------------------------------ multi-GPU combine: dense partials */
/* GroupByCombineOperator.mergeResults (GroupByCombineOperator.java:169-181) and
 * AggregationResultsBlockMerger (:33-45) merge per-segment results keyed by group VALUES.  Over table-level
 * dictionaries (ph_table_set_dictionary, identical on every GPU) a group is a dense id in
 * [0, num_groups), so the partial results of one GPU are a few dense device tables and the cross-GPU
 * merge is a plain reduction of those tables (RCCL reduce-scatter / all-reduce over xGMI, one op per
 * table: COUNT/SUM add, MIN/MAX min/max, HLL registers max = HyperLogLog.addAll).
 *
 *   ph_query_dense_layout   the tables of a query: count, per element type and reduce op
 *   ph_query_execute_dense  scans this GPU's segments into caller-allocated device tables (initialised
 *                           here), launching on the context's stream; nothing is copied to the host
 *   ph_dense_finalize       turns key shard [group_begin, group_end) of reduced tables (device pointers to
 *                           the shard's first group) into a ph_result, exactly like ph_query_execute's */
typedef enum {
  PH_REDUCE_SUM_I64 = 0, /* int64 add (COUNT, integer SUM) */
  PH_REDUCE_SUM_F64 = 1, /* float64 add (FLOAT/DOUBLE SUM; order-dependent within 1e-9 relative) */
  PH_REDUCE_MIN_I64 = 2, /* int64 min (MIN: integer values, or order keys of doubles) */
  PH_REDUCE_MAX_I64 = 3, /* int64 max (MAX) */
  PH_REDUCE_MAX_U32 = 4  /* uint32 max (DISTINCTCOUNTHLL registers) */
} ph_reduce_op;

#define PH_MAX_DENSE_TABLES 16
typedef struct {
  int64_t num_groups;                            /* dense key space (1 for aggregation-only queries) */
  int32_t num_tables;
  int32_t elems_per_group[PH_MAX_DENSE_TABLES];  /* table t: num_groups * elems_per_group[t] elements */
  int32_t reduce_op[PH_MAX_DENSE_TABLES];        /* ph_reduce_op */
  int32_t elem_bytes[PH_MAX_DENSE_TABLES];       /* 8 or 4 */
} ph_dense_layout;

int ph_query_dense_layout(ph_ctx* ctx, const ph_query* query, ph_segment* const* segments, int32_t num_segments,
                          ph_dense_layout* out);
int ph_query_execute_dense(ph_ctx* ctx, const ph_query* query, ph_segment* const* segments, int32_t num_segments,
                           void* const* device_tables, ph_exec_stats* stats);
int ph_dense_finalize(ph_ctx* ctx, const ph_query* query, ph_segment* const* segments, int32_t num_segments,
                      const void* const* device_tables, int64_t group_begin, int64_t group_end, ph_result** out);

/* ------------------------------------------------------------------ segment creation helper */
/* Raw forward index reader (BaseChunkForwardIndexReader / FixedByteChunkSVForwardIndexReader.getInt/getLong/
 * getFloat/getDouble over docs [0, num_docs)): decodes `buf` into num_docs native-endian values of `data_type`
 * (INT int32, LONG int64, FLOAT float, DOUBLE double) at `out`.  Host-only; what ph_segment_pin runs on a raw
 * column. */
int ph_raw_forward_index_read(const void* buf, uint64_t size, int32_t data_type, int32_t num_docs, void* out);

/* The V3 index_map reader the directory loader uses (SingleFileIndexDirectory.loadMap :213-247, keys split from the
 * right as ColumnIndexUtils.parseIndexMapKeys :33-45): the startOffset and size (magic included) of `column`'s
 * `index_id` buffer in columns.psf.  PH_ERR_BAD_QUERY when the map has no such entry; PH_ERR_INVALID_ARGUMENT when the
 * file is missing or malformed.  Host-only. */
int ph_index_map_lookup(const char* index_map_path, const char* column, const char* index_id, int64_t* start_offset,
                        int64_t* size);

/* FixedBitSVForwardIndexWriter: packs n dictIds with `bits` bits, MSB-first big-endian; out_size >=
 * (n*bits+7)/8 */
int ph_fixed_bit_pack(const int32_t* dict_ids, int64_t n, int32_t bits, uint8_t* out, uint64_t out_size);

/* Self-test hooks (FixedBitIntReaderTest-style parity checks, FixedBitIntReaderTest.java:43-81): unpack n values
 * of a packed fixed-bit stream on the device, writing dictIds to host memory `out`.
 *   ph_selftest_unpack         the per-doc gather routine (generic filter programs, value re-encoding, HLL)
 *   ph_selftest_unpack_staged  the scan kernels' staged tile decode (coalesced 16-byte loads -> LDS ->
 *                              one funnel shift per value) with `tile_words` 64-doc words per wave tile */
int ph_selftest_unpack(ph_ctx* ctx, const uint8_t* packed, uint64_t packed_size, int64_t n, int32_t bits,
                       int32_t* out);
int ph_selftest_unpack_staged(ph_ctx* ctx, const uint8_t* packed, uint64_t packed_size, int64_t n, int32_t bits,
                              int32_t tile_words, int32_t* out);

/* thread-local message of the last error on this thread */
const char* ph_last_error(void);
const char* ph_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PINOT_HIP_H */
