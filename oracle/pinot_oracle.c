/*
 * pinot_oracle.c -- CPU restatement of the reference path (TEST INFRASTRUCTURE ONLY; see
 * pinot_oracle.h).  Structure follows the reference loop for loop:
 *
 *   per segment task (GroupByCombineOperator.processSegments, GroupByCombineOperator.java:125-197)
 *     DocIdSetOperator.getNextBlock      (core/operator/DocIdSetOperator.java:59-86)   <= 10 000 docs
 *       SVScanDocIdIterator.next        (core/operator/dociditerators/SVScanDocIdIterator.java:76-98)
 *         256-doc batches: FixedBitSVForwardIndexReaderV2.readDictIds + PredicateEvaluator.applySV
 *     ProjectionOperator -> DataFetcher.readDictIds (per matched doc)
 *     DefaultGroupByExecutor.process    (DefaultGroupByExecutor.java:131-148)
 *       DictionaryBasedGroupKeyGenerator raw key = sum dictId_j * prod_{i<j} C_i (column 0 least
 *       significant, DictionaryBasedGroupKeyGenerator.java:283-313) ; first-seen group ids capped
 *       at numGroupsLimit (IntGroupIdMap.getGroupId :992-1017) ; INVALID_ID rows dropped.
 *       Sum/Min/Max/Count aggregateGroupBySV with double holders (SumAggregationFunction.java:207-240,
 *       CountAggregationFunction.java:104-154, Min/MaxAggregationFunction).
 *     DISTINCTCOUNTHLL: the reference collects the dictIds of the matched docs in a RoaringBitmap
 *       and offers dictionary.get(dictId) once per distinct id at extract time
 *       (DistinctCountHLLAggregationFunction.java:105-110,438-447).  HLL offer is idempotent and
 *       register-wise max, so offering each matched row's value yields identical registers; this
 *       restatement offers per row.
 *   merge: values-keyed table (IndexedTable.upsert, ConcurrentIndexedTable.java:44-81) -- here keyed
 *       by the mixed-radix key of table-level global ids (a bijection with the value tuple).
 */
#include "pinot_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ fixed-bit codec */
static const int FIRST_BIT_SET[256] = {
    /* PinotDataBitSet.FIRST_BIT_SET: number of leading zero bits in a byte value */
    8, 7, 6, 6, 5, 5, 5, 5, 4, 4, 4, 4, 4, 4, 4, 4, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3,
    2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2,
    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

int or_num_bits_per_value(int32_t max_value) {
  /* PinotDataBitSet.java:59-70 */
  if (max_value <= 1) return 1;
  int num_bits = 8;
  uint32_t v = (uint32_t)max_value;
  while (v > 0xFF) {
    v >>= 8;
    num_bits += 8;
  }
  return num_bits - FIRST_BIT_SET[v];
}

int64_t or_fixed_bit_num_bytes(int64_t n, int bits) { return (n * bits + 7) / 8; }

void or_fixed_bit_write(const int32_t* values, int64_t n, int bits, uint8_t* buf) {
  /* PinotDataBitSet.writeInt(int index, int numBitsPerValue, int value), PinotDataBitSet.java:138-165 */
  for (int64_t index = 0; index < n; index++) {
    int32_t value = values[index];
    int64_t bit_offset = index * bits;
    int64_t byte_offset = bit_offset / 8;
    int bit_in_first = (int)(bit_offset % 8);
    int first_byte = (int8_t)buf[byte_offset];
    int first_mask = 0xFF >> bit_in_first;
    int left = bits - (8 - bit_in_first);
    if (left <= 0) {
      first_mask &= 0xFF << -left;
      buf[byte_offset] = (uint8_t)((first_byte & ~first_mask) | (value << -left));
    } else {
      buf[byte_offset] = (uint8_t)((first_byte & ~first_mask) | (((uint32_t)value >> left) & first_mask));
      while (left > 8) {
        left -= 8;
        byte_offset++;
        buf[byte_offset] = (uint8_t)(value >> left);
      }
      byte_offset++;
      int last_byte = (int8_t)buf[byte_offset];
      buf[byte_offset] = (uint8_t)((last_byte & (0xFF >> left)) | (value << (8 - left)));
    }
  }
}

int32_t or_fixed_bit_read(const uint8_t* buf, int64_t index, int bits) {
  /* PinotDataBitSet.readInt, PinotDataBitSet.java:78-100 */
  int64_t bit_offset = index * bits;
  int64_t byte_offset = bit_offset / 8;
  int bit_in_first = (int)(bit_offset % 8);
  uint32_t cur = buf[byte_offset] & (0xFFu >> bit_in_first);
  int left = bits - (8 - bit_in_first);
  if (left <= 0) return (int32_t)(cur >> -left);
  while (left > 8) {
    byte_offset++;
    cur = (cur << 8) | buf[byte_offset];
    left -= 8;
  }
  return (int32_t)((cur << left) | ((uint32_t)buf[byte_offset + 1] >> (8 - left)));
}

void or_fixed_bit_read_range(const uint8_t* buf, int64_t start, int bits, int32_t length, int32_t* out) {
  /* PinotDataBitSet.readInt(startIndex, numBitsPerValue, length, buffer), PinotDataBitSet.java:102-136 */
  int64_t bit_offset = start * bits;
  int64_t byte_offset = bit_offset / 8;
  int bit_in_first = (int)(bit_offset % 8);
  uint32_t cur = buf[byte_offset] & (0xFFu >> bit_in_first);
  for (int32_t i = 0; i < length; i++) {
    if (bit_in_first == 8) {
      bit_in_first = 0;
      byte_offset++;
      cur = buf[byte_offset];
    }
    int left = bits - (8 - bit_in_first);
    if (left <= 0) {
      out[i] = (int32_t)(cur >> -left);
      bit_in_first = 8 + left;
      cur = cur & (0xFFu >> bit_in_first);
    } else {
      while (left > 8) {
        byte_offset++;
        cur = (cur << 8) | buf[byte_offset];
        left -= 8;
      }
      byte_offset++;
      uint32_t next = buf[byte_offset];
      out[i] = (int32_t)((cur << left) | (next >> (8 - left)));
      bit_in_first = left;
      cur = next & (0xFFu >> bit_in_first);
    }
  }
}

/* ------------------------------------------------------------------ HLL (clearspring 2.7.0) */
int32_t or_murmur_hash_long(int64_t data) {
  /* MurmurHash.hashLong(long): 32-bit arithmetic wraps as Java int */
  const uint32_t m = 0x5bd1e995u;
  const int r = 24;
  uint32_t h = 0;
  uint32_t k = (uint32_t)(int32_t)data * m;
  k ^= k >> r;
  h ^= k * m;
  k = (uint32_t)(int32_t)(data >> 32) * m;
  k ^= k >> r;
  h *= m;
  h ^= k * m;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

int32_t or_murmur_hash_bytes(const uint8_t* data, int32_t length, int32_t seed) {
  /* MurmurHash.hash(byte[] data, int length, int seed); Java bytes are signed */
  const uint32_t m = 0x5bd1e995u;
  const int r = 24;
  uint32_t h = (uint32_t)(seed ^ length);
  int32_t len4 = length >> 2;
  for (int32_t i = 0; i < len4; i++) {
    int32_t i4 = i << 2;
    uint32_t k = (uint32_t)(int32_t)(int8_t)data[i4 + 3];
    k = k << 8;
    k = k | (data[i4 + 2] & 0xff);
    k = k << 8;
    k = k | (data[i4 + 1] & 0xff);
    k = k << 8;
    k = k | (data[i4 + 0] & 0xff);
    k *= m;
    k ^= k >> r;
    k *= m;
    h *= m;
    h ^= k;
  }
  int32_t lenm = len4 << 2;
  int32_t left = length - lenm;
  if (left != 0) {
    if (left >= 3) h ^= (uint32_t)((int32_t)(int8_t)data[length - 3] << 16);
    if (left >= 2) h ^= (uint32_t)((int32_t)(int8_t)data[length - 2] << 8);
    if (left >= 1) h ^= (uint32_t)(int32_t)(int8_t)data[length - 1];
    h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

static int nlz32(uint32_t x) { return x == 0 ? 32 : __builtin_clz(x); }

void or_hll_offer_hashed(uint8_t* reg, int log2m, int32_t hashed) {
  /* HyperLogLog.offerHashed(int): j = h >>> (32-log2m);
   * r = numberOfLeadingZeros((h << log2m) | (1 << (log2m - 1)) + 1) + 1  ('+' binds before '|') */
  uint32_t h = (uint32_t)hashed;
  uint32_t j = h >> (32 - log2m);
  int r = nlz32((h << log2m) | ((1u << (log2m - 1)) + 1u)) + 1;
  if (reg[j] < r) reg[j] = (uint8_t)r;
}

static int64_t java_round(double x) {
  /* Math.round(double): floor(x + 0.5) with saturation */
  if (isnan(x)) return 0;
  double f = floor(x + 0.5);
  if (f >= 9.2233720368547758e18) return INT64_MAX;
  if (f <= -9.2233720368547758e18) return INT64_MIN;
  return (int64_t)f;
}

int64_t or_hll_cardinality(const uint8_t* reg, int log2m) {
  /* HyperLogLog.cardinality() with getAlphaMM(log2m, m) */
  int m = 1 << log2m;
  double sum = 0.0, zeros = 0.0;
  for (int j = 0; j < m; j++) {
    sum += 1.0 / (double)(1 << reg[j]);
    if (reg[j] == 0) zeros++;
  }
  double alpha_mm;
  switch (log2m) {
    case 4: alpha_mm = 0.673 * m * m; break;
    case 5: alpha_mm = 0.697 * m * m; break;
    case 6: alpha_mm = 0.709 * m * m; break;
    default: alpha_mm = (0.7213 / (1 + 1.079 / m)) * m * m;
  }
  double estimate = alpha_mm * (1 / sum);
  if (estimate <= (5.0 / 2.0) * m) return java_round(m * log(m / zeros));
  return java_round(estimate);
}

/* ------------------------------------------------------------------ hash map (u64 -> int) */
typedef struct {
  uint64_t* keys;
  int32_t* vals;
  int64_t cap;  /* power of two */
  int64_t size;
} u64map;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

static void map_init(u64map* m, int64_t cap) {
  int64_t c = 16;
  while (c < cap * 2) c <<= 1;
  m->cap = c;
  m->size = 0;
  m->keys = (uint64_t*)malloc(sizeof(uint64_t) * c);
  m->vals = (int32_t*)malloc(sizeof(int32_t) * c);
  for (int64_t i = 0; i < c; i++) m->vals[i] = -1;
}

static void map_free(u64map* m) {
  free(m->keys);
  free(m->vals);
}

static void map_grow(u64map* m) {
  u64map n;
  map_init(&n, m->cap);
  for (int64_t i = 0; i < m->cap; i++) {
    if (m->vals[i] < 0) continue;
    uint64_t p = mix64(m->keys[i]) & (n.cap - 1);
    while (n.vals[p] >= 0) p = (p + 1) & (n.cap - 1);
    n.keys[p] = m->keys[i];
    n.vals[p] = m->vals[i];
  }
  n.size = m->size;
  map_free(m);
  *m = n;
}

/* returns existing id, or inserts next id when size < limit, else -1 (GroupKeyGenerator.INVALID_ID) */
static int32_t map_get_or_put(u64map* m, uint64_t key, int64_t limit) {
  uint64_t p = mix64(key) & (m->cap - 1);
  while (m->vals[p] >= 0) {
    if (m->keys[p] == key) return m->vals[p];
    p = (p + 1) & (m->cap - 1);
  }
  if (m->size >= limit) return -1;
  m->keys[p] = key;
  m->vals[p] = (int32_t)m->size++;
  if (m->size * 2 > m->cap) map_grow(m);
  return (int32_t)(m->size - 1);
}

/* ------------------------------------------------------------------ per-segment execution */
#define SCAN_BATCH 256   /* BlockDocIdIterator.OPTIMAL_ITERATOR_BATCH_SIZE (core/common/BlockDocIdIterator.java:49) */
#define DOC_BLOCK 10000  /* DocIdSetPlanNode.MAX_DOC_PER_CALL (core/plan/DocIdSetPlanNode.java:29) */

static int32_t read_dict_id(const or_column* c, int32_t doc) {
  if (c->fwd) return or_fixed_bit_read(c->fwd, doc, c->bits);
  /* SortedIndexReaderImpl.getDictId: binary search over the (start,end) ranges */
  int32_t lo = 0, hi = c->cardinality - 1;
  while (lo < hi) {
    int32_t mid = (lo + hi + 1) >> 1;
    if (c->sorted[2 * mid] <= doc) lo = mid; else hi = mid - 1;
  }
  return lo;
}

static int eval_filter_doc(const or_query* q, const or_segment* s, int32_t doc, int64_t* scanned) {
  int stack[64];
  int sp = 0;
  for (int i = 0; i < q->num_filter_ops; i++) {
    const or_filter_op* op = &q->filter[i];
    switch (op->op) {
      case OR_F_LEAF: {
        const or_column* c = &s->columns[op->arg];
        if (op->is_scan) (*scanned)++;
        stack[sp++] = op->match[read_dict_id(c, doc)] != 0;
        break;
      }
      case OR_F_AND: {
        if (op->is_scan) {
          /* applyAnd (AndDocIdSet.java:168-170, SVScanDocIdIterator.applyAnd :115-142): the doc reaches the first
           * scan if every index-based child matched, scan i+1 if it also passed scans 1..i */
          const int nidx = op->is_scan >> 8, nscan = op->is_scan & 255;
          const int* kid = stack + sp - op->arg;
          int ok = 1;
          for (int k = 0; k < nidx; k++) ok &= kid[k];
          if (ok) {
            int fed = 1;
            for (int k = 0; k + 1 < nscan && kid[nidx + k]; k++) fed++;
            *scanned += fed;
          }
        }
        int v = 1;
        for (int k = 0; k < op->arg; k++) v &= stack[--sp];
        stack[sp++] = v;
        break;
      }
      case OR_F_OR: {
        int v = 0;
        for (int k = 0; k < op->arg; k++) v |= stack[--sp];
        stack[sp++] = v;
        break;
      }
      case OR_F_NOT: stack[sp - 1] = !stack[sp - 1]; break;
      case OR_F_ALL: stack[sp++] = 1; break;
      case OR_F_NONE: stack[sp++] = 0; break;
    }
  }
  return stack[0];
}

typedef struct {
  u64map map;          /* local raw key -> group id */
  uint64_t* gkeys;     /* group id -> global key */
  double* aggs;        /* [group][num_aggs] */
  uint8_t* hll;        /* [group][num_hll][m] */
  int64_t ngroups, cap;
  int64_t docs_scanned, in_filter, post_filter;
  int limit_reached;
} seg_result;

static void seg_grow(seg_result* r, int nagg, int hll_bytes) {
  int64_t nc = r->cap ? r->cap * 2 : 1024;
  r->gkeys = (uint64_t*)realloc(r->gkeys, sizeof(uint64_t) * nc);
  r->aggs = (double*)realloc(r->aggs, sizeof(double) * nc * (nagg ? nagg : 1));
  if (hll_bytes) {
    r->hll = (uint8_t*)realloc(r->hll, (size_t)nc * hll_bytes);
    memset(r->hll + (size_t)r->cap * hll_bytes, 0, (size_t)(nc - r->cap) * hll_bytes);
  }
  r->cap = nc;
}

static void agg_init(const or_query* q, double* a) {
  for (int k = 0; k < q->num_aggs; k++) {
    switch (q->agg_fn[k]) {
      case OR_AGG_MIN: a[k] = INFINITY; break;   /* MinAggregationFunction default +inf */
      case OR_AGG_MAX: a[k] = -INFINITY; break;  /* MaxAggregationFunction default -inf */
      default: a[k] = 0.0;
    }
  }
}

static int32_t hll_hash(const or_column* c, int32_t dict_id) {
  if (c->hash_longs) return or_murmur_hash_long(c->hash_longs[dict_id]);
  return c->hash_ints[dict_id];
}

/* DataFetcher.readDoubleValues (DataFetcher.java:529-539) of the aggregated argument; a 2-operand expression is
 * evaluated in double like the reference's TransformFunction.transformToDoubleValuesSV */
static double agg_value(const or_query* q, const or_segment* s, int k, int32_t doc) {
  const or_column* ca = &s->columns[q->agg_col[k]];
  const double a = ca->values[read_dict_id(ca, doc)];
  const int op = q->agg_op ? q->agg_op[k] : 0;
  if (!op) return a;
  const or_column* cb = &s->columns[q->agg_col2[k]];
  const double b = cb->values[read_dict_id(cb, doc)];
  return op == 1 ? (1.0 * a) * b : (op == 2 ? a - b : a + b);
}

static void run_segment(const or_query* q, const or_segment* s, seg_result* r) {
  const int nagg = q->num_aggs;
  const int m = 1 << q->log2m;
  int nhll = 0;
  for (int k = 0; k < nagg; k++) nhll += q->agg_fn[k] == OR_AGG_HLL;
  const int hll_bytes = nhll * m;
  memset(r, 0, sizeof(*r));

  /* key space: local raw key over this segment's cardinalities (column 0 least significant) */
  int64_t card_product = 1;
  for (int g = 0; g < q->num_group_by; g++) card_product *= s->columns[q->group_cols[g]].cardinality;
  map_init(&r->map, 1024);

  int32_t* doc_ids = (int32_t*)malloc(sizeof(int32_t) * (DOC_BLOCK + SCAN_BATCH));
  int32_t* dict_buf = (int32_t*)malloc(sizeof(int32_t) * SCAN_BATCH);
  int single_scan = q->num_filter_ops == 1 && q->filter[0].op == OR_F_LEAF &&
                    s->columns[q->filter[0].arg].fwd != NULL;
  int32_t next_doc = 0;
  const int32_t n = s->num_docs;
  int no_group = q->num_group_by == 0;
  if (no_group) {
    seg_grow(r, nagg, hll_bytes);
    r->ngroups = 1;
    r->gkeys[0] = 0;
    agg_init(q, r->aggs);
  }
  int32_t pending = 0; /* docs carried over from the last 256 batch beyond the block limit */
  int32_t carry[SCAN_BATCH];
  while (1) {
    /* DocIdSetOperator.getNextBlock: collect up to DOC_BLOCK matching docs */
    int32_t cnt = 0;
    for (int32_t i = 0; i < pending; i++) doc_ids[cnt++] = carry[i];
    pending = 0;
    while (cnt < DOC_BLOCK && next_doc < n) {
      int32_t lim = n - next_doc < SCAN_BATCH ? n - next_doc : SCAN_BATCH;
      if (q->num_filter_ops == 0) {
        for (int32_t i = 0; i < lim; i++) doc_ids[cnt++] = next_doc + i;
      } else if (single_scan) {
        /* SVScanDocIdIterator.next: readDictIds(contiguous batch) + applySV compaction */
        const or_filter_op* op = &q->filter[0];
        const or_column* c = &s->columns[op->arg];
        or_fixed_bit_read_range(c->fwd, next_doc, c->bits, lim, dict_buf);
        if (op->is_scan) r->in_filter += lim;  /* an index-based leaf read through its forward index scans nothing */
        for (int32_t i = 0; i < lim; i++)
          if (op->match[dict_buf[i]]) doc_ids[cnt++] = next_doc + i;
      } else {
        for (int32_t i = 0; i < lim; i++)
          if (eval_filter_doc(q, s, next_doc + i, &r->in_filter)) doc_ids[cnt++] = next_doc + i;
      }
      next_doc += lim;
    }
    if (cnt > DOC_BLOCK) {
      pending = cnt - DOC_BLOCK;
      memcpy(carry, doc_ids + DOC_BLOCK, sizeof(int32_t) * pending);
      cnt = DOC_BLOCK;
    }
    if (cnt == 0) break;
    r->docs_scanned += cnt;
    /* projection + group-by executor, doc by doc over the block */
    for (int32_t i = 0; i < cnt; i++) {
      int32_t doc = doc_ids[i];
      int64_t gid = 0;
      if (!no_group) {
        uint64_t raw = 0;
        for (int g = q->num_group_by - 1; g >= 0; g--) {
          const or_column* c = &s->columns[q->group_cols[g]];
          raw = raw * (uint64_t)c->cardinality + (uint64_t)read_dict_id(c, doc);
        }
        int32_t id = map_get_or_put(&r->map, raw, q->num_groups_limit);
        if (id < 0) {
          r->limit_reached = 1;
          continue; /* INVALID_ID: DoubleGroupByResultHolder ignores it */
        }
        if (id >= r->ngroups) {
          if (id >= r->cap) seg_grow(r, nagg, hll_bytes);
          /* global key from global ids */
          uint64_t gk = 0;
          for (int g = q->num_group_by - 1; g >= 0; g--) {
            const or_column* c = &s->columns[q->group_cols[g]];
            gk = gk * (uint64_t)q->group_global_card[g] + (uint64_t)c->global_ids[read_dict_id(c, doc)];
          }
          r->gkeys[id] = gk;
          agg_init(q, r->aggs + (int64_t)id * nagg);
          r->ngroups = id + 1;
        }
        gid = id;
      }
      double* a = r->aggs + gid * nagg;
      int h = 0;
      for (int k = 0; k < nagg; k++) {
        int32_t col = q->agg_col[k];
        switch (q->agg_fn[k]) {
          case OR_AGG_COUNT: a[k] += 1.0; break;
          case OR_AGG_SUM: a[k] += agg_value(q, s, k, doc); break;
          case OR_AGG_MIN: {
            double v = agg_value(q, s, k, doc);
            if (v < a[k]) a[k] = v;
            break;
          }
          case OR_AGG_MAX: {
            double v = agg_value(q, s, k, doc);
            if (v > a[k]) a[k] = v;
            break;
          }
          case OR_AGG_HLL: {
            const or_column* c = &s->columns[col];
            or_hll_offer_hashed(r->hll + (size_t)gid * hll_bytes + (size_t)h * m, q->log2m,
                                hll_hash(c, read_dict_id(c, doc)));
            h++;
            break;
          }
        }
      }
    }
  }
  /* numEntriesScannedPostFilter = numDocsScanned * #distinct projected columns */
  int ncols_proj = 0;
  {
    int seen[256] = {0};
    for (int g = 0; g < q->num_group_by; g++)
      if (!seen[q->group_cols[g]]) { seen[q->group_cols[g]] = 1; ncols_proj++; }
    for (int k = 0; k < nagg; k++) {
      if (q->agg_col[k] >= 0 && !seen[q->agg_col[k]]) { seen[q->agg_col[k]] = 1; ncols_proj++; }
      if (q->agg_op && q->agg_op[k] && !seen[q->agg_col2[k]]) { seen[q->agg_col2[k]] = 1; ncols_proj++; }
    }
  }
  r->post_filter = r->docs_scanned * ncols_proj;
  /* GroupByOperator.java:111: numGroupsLimitReached = getNumGroups() >= numGroupsLimit */
  if (!no_group && r->ngroups >= q->num_groups_limit) r->limit_reached = 1;
  (void)card_product;
  free(doc_ids);
  free(dict_buf);
}

/* ------------------------------------------------------------------ combine */
typedef struct {
  const or_query* q;
  const or_segment* segs;
  int32_t nseg;
  int32_t next;
  pthread_mutex_t lock;
  u64map table;
  uint64_t* keys;
  double* aggs;
  uint8_t* hll;
  int64_t n, cap;
  int hll_bytes;
  int64_t docs_scanned, in_filter, post_filter, total_docs;
  int limit_reached;
} combine_ctx;

static void merge_locked(combine_ctx* c, seg_result* r) {
  const or_query* q = c->q;
  const int nagg = q->num_aggs;
  const int m = 1 << q->log2m;
  for (int64_t g = 0; g < r->ngroups; g++) {
    int32_t id = map_get_or_put(&c->table, r->gkeys[g], INT64_MAX);
    if (id >= c->cap) {
      int64_t nc = c->cap ? c->cap * 2 : 1024;
      while (nc <= id) nc *= 2;
      c->keys = (uint64_t*)realloc(c->keys, sizeof(uint64_t) * nc);
      c->aggs = (double*)realloc(c->aggs, sizeof(double) * nc * (nagg ? nagg : 1));
      if (c->hll_bytes) {
        c->hll = (uint8_t*)realloc(c->hll, (size_t)nc * c->hll_bytes);
        memset(c->hll + (size_t)c->cap * c->hll_bytes, 0, (size_t)(nc - c->cap) * c->hll_bytes);
      }
      c->cap = nc;
    }
    double* dst = c->aggs + (int64_t)id * nagg;
    const double* src = r->aggs + g * nagg;
    if (id >= c->n) {
      c->keys[id] = r->gkeys[g];
      memcpy(dst, src, sizeof(double) * nagg);
      if (c->hll_bytes) memcpy(c->hll + (size_t)id * c->hll_bytes, r->hll + (size_t)g * c->hll_bytes, c->hll_bytes);
      c->n = id + 1;
      continue;
    }
    /* AggregationFunction.merge */
    for (int k = 0; k < nagg; k++) {
      switch (q->agg_fn[k]) {
        case OR_AGG_COUNT:
        case OR_AGG_SUM: dst[k] += src[k]; break;
        case OR_AGG_MIN: if (src[k] < dst[k]) dst[k] = src[k]; break;
        case OR_AGG_MAX: if (src[k] > dst[k]) dst[k] = src[k]; break;
        default: break;
      }
    }
    if (c->hll_bytes) {
      uint8_t* d = c->hll + (size_t)id * c->hll_bytes;
      const uint8_t* s = r->hll + (size_t)g * c->hll_bytes;
      for (int b = 0; b < c->hll_bytes; b++) if (s[b] > d[b]) d[b] = s[b];  /* HyperLogLog.addAll */
    }
  }
  (void)m;
  c->docs_scanned += r->docs_scanned;
  c->in_filter += r->in_filter;
  c->post_filter += r->post_filter;
  c->limit_reached |= r->limit_reached;
}

static void* worker(void* arg) {
  combine_ctx* c = (combine_ctx*)arg;
  while (1) {
    int32_t i = __atomic_fetch_add(&c->next, 1, __ATOMIC_RELAXED);
    if (i >= c->nseg) break;
    seg_result r;
    run_segment(c->q, &c->segs[i], &r);
    pthread_mutex_lock(&c->lock);
    merge_locked(c, &r);
    pthread_mutex_unlock(&c->lock);
    map_free(&r.map);
    free(r.gkeys);
    free(r.aggs);
    free(r.hll);
  }
  return NULL;
}

int or_execute(const or_query* q, const or_segment* segs, int32_t nseg, int32_t nthreads, or_result* out) {
  combine_ctx c;
  memset(&c, 0, sizeof(c));
  c.q = q;
  c.segs = segs;
  c.nseg = nseg;
  int nhll = 0;
  for (int k = 0; k < q->num_aggs; k++) nhll += q->agg_fn[k] == OR_AGG_HLL;
  c.hll_bytes = nhll * (1 << q->log2m);
  pthread_mutex_init(&c.lock, NULL);
  map_init(&c.table, 1024);
  for (int i = 0; i < nseg; i++) c.total_docs += segs[i].num_docs;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > nseg) nthreads = nseg > 0 ? nseg : 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &c);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  map_free(&c.table);
  pthread_mutex_destroy(&c.lock);
  memset(out, 0, sizeof(*out));
  out->num_groups = c.n;
  out->keys = c.keys;
  out->aggs = c.aggs;
  out->hll = c.hll;
  out->num_hll = nhll;
  out->num_docs_scanned = c.docs_scanned;
  out->num_entries_scanned_in_filter = c.in_filter;
  out->num_entries_scanned_post_filter = c.post_filter;
  out->num_total_docs = c.total_docs;
  out->num_groups_limit_reached = c.limit_reached;
  if (q->num_group_by == 0 && c.n == 0) {
    /* aggregation-only over zero segments: one default row */
    out->num_groups = 1;
    out->keys = (uint64_t*)calloc(1, sizeof(uint64_t));
    out->aggs = (double*)malloc(sizeof(double) * (q->num_aggs ? q->num_aggs : 1));
    agg_init(q, out->aggs);
    if (c.hll_bytes) out->hll = (uint8_t*)calloc(1, c.hll_bytes);
  }
  return 0;
}

void or_result_free(or_result* r) {
  free(r->keys);
  free(r->aggs);
  free(r->hll);
  memset(r, 0, sizeof(*r));
}
