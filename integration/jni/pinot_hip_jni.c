/* pinot_hip_jni.c -- JNI shim between org.apache.pinot.core.gpu.PinotHipJni and libpinot_hip.so (include/pinot_hip.h).
 *
 * Not built in this repository (the image has no JDK, hence no jni.h); a maintainer builds it next to the library:
 *   cc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude integration/jni/pinot_hip_jni.c \
 *      -Lpinot_amd -lpinot_hip -o libpinot_hip_jni.so
 * Buffers cross as direct ByteBuffers (no copies); a query crosses as one int[] descriptor plus the strings it
 * indexes (layout in PinotHipJni.queryExecute), decoded here into the ph_query structs.  Every non-zero status
 * becomes a Java exception carrying ph_last_error(): PH_ERR_BAD_QUERY -> BadQueryRequestException
 * (PredicateEvaluatorProvider.java:92-95), PH_ERR_UNSUPPORTED -> UnsupportedOperationException (the plan maker falls
 * back to the CPU plan), PH_ERR_CANCELLED -> EarlyTerminationException (BaseOperator.java:39), else RuntimeException.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pinot_hip.h"

static int throw_ph(JNIEnv* env, int rc) {
  if (rc == PH_OK) return 0;
  const char* cls = rc == PH_ERR_BAD_QUERY     ? "org/apache/pinot/spi/exception/BadQueryRequestException"
                    : rc == PH_ERR_UNSUPPORTED ? "java/lang/UnsupportedOperationException"
                    : rc == PH_ERR_CANCELLED   ? "org/apache/pinot/spi/exception/EarlyTerminationException"
                                               : "java/lang/RuntimeException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, ph_last_error());
  return 1;
}

static void throw_illegal(JNIEnv* env, const char* msg);

#define FN(name) Java_org_apache_pinot_core_gpu_PinotHipJni_##name
#define PTR(x) ((void*)(intptr_t)(x))

JNIEXPORT jlong JNICALL FN(ctxCreate)(JNIEnv* env, jclass c, jint device) {
  ph_ctx* ctx = NULL;
  throw_ph(env, ph_ctx_create(device, &ctx));
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT jlong JNICALL FN(ctxCreateMulti)(JNIEnv* env, jclass c, jintArray devices) {
  ph_ctx* ctx = NULL;
  const jsize n = devices ? (*env)->GetArrayLength(env, devices) : 0;
  /* the whole ordinal list goes to the library unchanged (it rejects n > 64 itself); never a truncated set */
  jint* d = n ? (*env)->GetIntArrayElements(env, devices, NULL) : NULL;
  if (n && !d) return 0; /* OutOfMemoryError pending */
  int32_t* ords = (int32_t*)calloc((size_t)(n ? n : 1), sizeof(int32_t));
  if (!ords) {
    if (d) (*env)->ReleaseIntArrayElements(env, devices, d, JNI_ABORT);
    throw_illegal(env, "out of memory");
    return 0;
  }
  for (jsize i = 0; i < n; ++i) ords[i] = (int32_t)d[i];
  if (d) (*env)->ReleaseIntArrayElements(env, devices, d, JNI_ABORT);
  throw_ph(env, ph_ctx_create_multi(ords, (int32_t)n, &ctx));
  free(ords);
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL FN(ctxDestroy)(JNIEnv* env, jclass c, jlong ctx) { throw_ph(env, ph_ctx_destroy(PTR(ctx))); }

/* Strings of a Java String[] as UTF-8 for the duration of one call.  The element references are local refs held in
 * `refs` (the caller brackets the call in Push/PopLocalFrame, so many strings never overflow the local-reference
 * table); a null element stays NULL. */
typedef struct {
  jsize n;
  jstring* refs;
  const char** strs;
} utf_strings;

static int utf_strings_get(JNIEnv* env, jobjectArray arr, utf_strings* u) {
  u->n = arr ? (*env)->GetArrayLength(env, arr) : 0;
  u->refs = (jstring*)calloc((size_t)(u->n ? u->n : 1), sizeof(jstring));
  u->strs = (const char**)calloc((size_t)(u->n ? u->n : 1), sizeof(char*));
  if (!u->refs || !u->strs) return 0;
  for (jsize i = 0; i < u->n; ++i) {
    u->refs[i] = (jstring)(*env)->GetObjectArrayElement(env, arr, i);
    u->strs[i] = u->refs[i] ? (*env)->GetStringUTFChars(env, u->refs[i], NULL) : NULL;
    if (u->refs[i] && !u->strs[i]) return 0;  /* OutOfMemoryError pending */
  }
  return 1;
}

static void utf_strings_release(JNIEnv* env, utf_strings* u) {
  for (jsize i = 0; u->refs && u->strs && i < u->n; ++i)
    if (u->refs[i] && u->strs[i]) (*env)->ReleaseStringUTFChars(env, u->refs[i], u->strs[i]);
  free(u->refs);
  free(u->strs);
}

static void throw_illegal(JNIEnv* env, const char* msg) {
  jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
  if (c) (*env)->ThrowNew(env, c, msg);
}

/* ImmutableSegmentLoader.load -> pin the segment's directory (ph_segment_load_dir); columns == null: all */
JNIEXPORT jlong JNICALL FN(segmentLoadDir)(JNIEnv* env, jclass c, jlong ctx, jstring dir, jobjectArray columns) {
  const jsize n = columns ? (*env)->GetArrayLength(env, columns) : 0;
  if ((*env)->PushLocalFrame(env, n + 16) != 0) return 0;
  const char* d = (*env)->GetStringUTFChars(env, dir, NULL);
  utf_strings cols = {0, NULL, NULL};
  ph_segment* seg = NULL;
  int rc = PH_ERR_INVALID_ARGUMENT;
  if (d && utf_strings_get(env, columns, &cols)) {
    rc = ph_segment_load_dir(PTR(ctx), d, n ? cols.strs : NULL, (int32_t)n, &seg);
  }
  utf_strings_release(env, &cols);
  if (d) (*env)->ReleaseStringUTFChars(env, dir, d);
  (*env)->PopLocalFrame(env, NULL);
  if (!(*env)->ExceptionCheck(env)) throw_ph(env, rc);
  return (jlong)(intptr_t)seg;
}

JNIEXPORT void JNICALL FN(segmentUnpin)(JNIEnv* env, jclass c, jlong seg) { throw_ph(env, ph_segment_unpin(PTR(seg))); }

JNIEXPORT jlong JNICALL FN(segmentDeviceBytes)(JNIEnv* env, jclass c, jlong seg) {
  return ph_segment_device_bytes(PTR(seg));
}

JNIEXPORT jint JNICALL FN(segmentDevice)(JNIEnv* env, jclass c, jlong seg) { return ph_segment_device(PTR(seg)); }

/* table-level dictionary of a group-by column (sorted values, fixed width, direct buffer) */
JNIEXPORT void JNICALL FN(tableSetDictionary)(JNIEnv* env, jclass c, jlong ctx, jstring column, jint dataType,
                                              jobject values, jlong count, jint entrySize) {
  const char* col = (*env)->GetStringUTFChars(env, column, NULL);
  const int rc = ph_table_set_dictionary(PTR(ctx), col, dataType, (*env)->GetDirectBufferAddress(env, values), count,
                                         entrySize);
  (*env)->ReleaseStringUTFChars(env, column, col);
  throw_ph(env, rc);
}

JNIEXPORT void JNICALL FN(tableSetColumnType)(JNIEnv* env, jclass c, jlong ctx, jstring column, jint dataType) {
  const char* col = (*env)->GetStringUTFChars(env, column, NULL);
  const int rc = ph_table_set_column_type(PTR(ctx), col, dataType);
  (*env)->ReleaseStringUTFChars(env, column, col);
  throw_ph(env, rc);
}

/* Query descriptor (ints; string operands are indices into `strs`, -1 = NULL):
 *   [numFilterNodes, filterRoot, numPredicates, numGroupBy, numAggregations,
 *    per filter node: type, numChildren, predicate, child...,
 *    per predicate: type, column, numValues, value..., lower, upper, lowerInclusive, upperInclusive,
 *    per group-by column: column,
 *    per aggregation: type, column, log2m, column2, exprOp,
 *    optional: numOrderBy, (kind, index, asc) x numOrderBy, limit, minSegmentGroupTrimSize]
 * decoded into `q`; the arrays it points into are owned by `b` (query_bufs_free).  Returns 0, or -1 for a malformed
 * descriptor (every read is bounds-checked). */
typedef struct {
  ph_filter_node* nodes;
  ph_predicate* preds;
  const char** gby;
  ph_aggregation* aggs;
  ph_order_by* order;
  int32_t* ints;
  const char** vals;
} query_bufs;

static void query_bufs_free(query_bufs* b) {
  free(b->nodes); free(b->preds); free(b->gby); free(b->aggs); free(b->ints); free(b->vals); free(b->order);
}

static int decode_query(const jint* desc, jsize nd, const char** strs, jsize ns, ph_query* q, query_bufs* b) {
#define S(i) ((i) >= 0 && (i) < ns ? strs[(i)] : NULL)
#define NEXT(dst)             \
  do {                        \
    if (k >= nd) return -1;   \
    (dst) = desc[k++];        \
  } while (0)
  int k = 0, tmp = 0;
  memset(q, 0, sizeof *q);
  memset(b, 0, sizeof *b);
  NEXT(q->num_filter_nodes);
  NEXT(q->filter_root);
  NEXT(q->num_predicates);
  NEXT(q->num_group_by);
  NEXT(q->num_aggregations);
  /* every entity takes at least one descriptor int, so a count beyond nd is malformed */
  if (q->num_filter_nodes < 0 || q->num_predicates < 0 || q->num_group_by < 0 || q->num_aggregations < 0 ||
      q->num_filter_nodes > nd || q->num_predicates > nd || q->num_group_by > nd || q->num_aggregations > nd)
    return -1;
  b->nodes = (ph_filter_node*)calloc((size_t)q->num_filter_nodes + 1, sizeof(ph_filter_node));
  b->preds = (ph_predicate*)calloc((size_t)q->num_predicates + 1, sizeof(ph_predicate));
  b->gby = (const char**)calloc((size_t)q->num_group_by + 1, sizeof(char*));
  b->aggs = (ph_aggregation*)calloc((size_t)q->num_aggregations + 1, sizeof(ph_aggregation));
  b->ints = (int32_t*)calloc((size_t)nd + 1, sizeof(int32_t)); /* children lists live here (<= nd entries) */
  b->vals = (const char**)calloc((size_t)nd + 1, sizeof(char*));
  if (!b->nodes || !b->preds || !b->gby || !b->aggs || !b->ints || !b->vals) return -1;
  int ki = 0, kv = 0;
  for (int i = 0; i < q->num_filter_nodes; ++i) {
    NEXT(b->nodes[i].type);
    NEXT(b->nodes[i].num_children);
    NEXT(b->nodes[i].predicate);
    if (b->nodes[i].num_children < 0 || b->nodes[i].num_children > nd - k) return -1;
    b->nodes[i].children = b->ints + ki;
    for (int j = 0; j < b->nodes[i].num_children; ++j) NEXT(b->ints[ki++]);
  }
  for (int i = 0; i < q->num_predicates; ++i) {
    NEXT(b->preds[i].type);
    NEXT(tmp);
    b->preds[i].column = S(tmp);
    NEXT(b->preds[i].num_values);
    if (b->preds[i].num_values < 0 || b->preds[i].num_values > nd - k) return -1;
    b->preds[i].values = b->vals + kv;
    for (int j = 0; j < b->preds[i].num_values; ++j) {
      NEXT(tmp);
      b->vals[kv++] = S(tmp);
    }
    NEXT(tmp);
    b->preds[i].lower = S(tmp);
    NEXT(tmp);
    b->preds[i].upper = S(tmp);
    NEXT(b->preds[i].lower_inclusive);
    NEXT(b->preds[i].upper_inclusive);
  }
  for (int i = 0; i < q->num_group_by; ++i) {
    NEXT(tmp);
    b->gby[i] = S(tmp);
  }
  for (int i = 0; i < q->num_aggregations; ++i) {
    NEXT(b->aggs[i].type);
    NEXT(tmp);
    b->aggs[i].column = S(tmp);
    NEXT(b->aggs[i].log2m);
    NEXT(tmp);
    b->aggs[i].column2 = S(tmp);
    NEXT(b->aggs[i].expr_op);
  }
  if (k < nd) { /* optional trailing block: ORDER BY + LIMIT + minSegmentGroupTrimSize [+ skipStarTree] */
    NEXT(q->num_order_by);
    if (q->num_order_by < 0 || q->num_order_by > nd - k) return -1;
    b->order = (ph_order_by*)calloc((size_t)q->num_order_by + 1, sizeof(ph_order_by));
    if (!b->order) return -1;
    for (int i = 0; i < q->num_order_by; ++i) {
      NEXT(b->order[i].kind);
      NEXT(b->order[i].index);
      NEXT(b->order[i].asc);
    }
    NEXT(q->limit);
    NEXT(q->min_segment_group_trim_size);
    q->order_by = b->order;
    if (k < nd) NEXT(q->skip_star_tree); /* QueryContext.isSkipStarTree() */
  }
  /* indices inside the query (children, predicates, root) are range-checked by the library itself */
  q->filter_nodes = b->nodes;
  q->predicates = b->preds;
  q->group_by = b->gby;
  q->aggregations = b->aggs;
  return 0;
#undef NEXT
#undef S
}

JNIEXPORT jlong JNICALL FN(queryExecute)(JNIEnv* env, jclass c, jlong ctx, jintArray descArr, jobjectArray strArr,
                                         jlong numGroupsLimit, jlong endTimeMs, jlongArray segArr) {
  const jsize nd = (*env)->GetArrayLength(env, descArr);
  const jsize ns0 = strArr ? (*env)->GetArrayLength(env, strArr) : 0;
  if ((*env)->PushLocalFrame(env, ns0 + 16) != 0) return 0;
  jint* desc = (*env)->GetIntArrayElements(env, descArr, NULL);
  utf_strings us = {0, NULL, NULL};
  const int strs_ok = utf_strings_get(env, strArr, &us);
  ph_query q;
  query_bufs qb;
  memset(&qb, 0, sizeof qb);
  ph_result* res = NULL;
  int rc = PH_ERR_INVALID_ARGUMENT;
  if (desc && strs_ok) {
    if (decode_query(desc, nd, us.strs, us.n, &q, &qb) != 0) {
      throw_illegal(env, "malformed GPU query descriptor");
    } else {
      q.num_groups_limit = numGroupsLimit;
      q.end_time_ms = endTimeMs;
      const jsize nseg = (*env)->GetArrayLength(env, segArr);
      jlong* segs = (*env)->GetLongArrayElements(env, segArr, NULL);
      ph_segment** sp = (ph_segment**)calloc((size_t)(nseg ? nseg : 1), sizeof(ph_segment*));
      if (segs && sp) {
        for (jsize i = 0; i < nseg; ++i) sp[i] = (ph_segment*)PTR(segs[i]);
        rc = ph_query_execute(PTR(ctx), &q, sp, (int32_t)nseg, &res);
      }
      free(sp);
      if (segs) (*env)->ReleaseLongArrayElements(env, segArr, segs, JNI_ABORT);
    }
  }
  query_bufs_free(&qb);
  utf_strings_release(env, &us);
  if (desc) (*env)->ReleaseIntArrayElements(env, descArr, desc, JNI_ABORT);
  (*env)->PopLocalFrame(env, NULL);
  if (!(*env)->ExceptionCheck(env)) throw_ph(env, rc);
  return (jlong)(intptr_t)res;
}

/* ph_filter_execute over one segment (GpuFilterOperator): the doc bitmap straight into the Java long[] (bit i of word
 * w = doc 64 w + i: the java.util.BitSet / BitSetUtil.bitmapOf layout), or the count alone when docWords is null;
 * statsOut = {matching docs, numEntriesScannedInFilter} */
JNIEXPORT jlong JNICALL FN(filterExecute)(JNIEnv* env, jclass c, jlong ctx, jintArray descArr, jobjectArray strArr,
                                          jlong endTimeMs, jlong segment, jlongArray wordsArr, jlongArray statsArr) {
  const jsize nd = (*env)->GetArrayLength(env, descArr);
  const jsize ns0 = strArr ? (*env)->GetArrayLength(env, strArr) : 0;
  if ((*env)->PushLocalFrame(env, ns0 + 16) != 0) return 0;
  jint* desc = (*env)->GetIntArrayElements(env, descArr, NULL);
  utf_strings us = {0, NULL, NULL};
  const int strs_ok = utf_strings_get(env, strArr, &us);
  ph_query q;
  query_bufs qb;
  memset(&qb, 0, sizeof qb);
  ph_exec_stats st;
  memset(&st, 0, sizeof st);
  int rc = PH_ERR_INVALID_ARGUMENT;
  if (desc && strs_ok) {
    if (decode_query(desc, nd, us.strs, us.n, &q, &qb) != 0) {
      throw_illegal(env, "malformed GPU filter descriptor");
    } else {
      q.end_time_ms = endTimeMs;
      const jsize nw = wordsArr ? (*env)->GetArrayLength(env, wordsArr) : 0;
      /* critical section: the library writes the words in place (one D2H copy, no JNI copy-back) */
      jlong* words = wordsArr ? (jlong*)(*env)->GetPrimitiveArrayCritical(env, wordsArr, NULL) : NULL;
      if (!wordsArr || words) {
        rc = ph_filter_execute(PTR(ctx), &q, (ph_segment*)PTR(segment), (uint64_t*)words, (uint64_t)nw, &st);
        if (words) (*env)->ReleasePrimitiveArrayCritical(env, wordsArr, words, 0);
      }
    }
  }
  query_bufs_free(&qb);
  utf_strings_release(env, &us);
  if (desc) (*env)->ReleaseIntArrayElements(env, descArr, desc, JNI_ABORT);
  (*env)->PopLocalFrame(env, NULL);
  if ((*env)->ExceptionCheck(env) || throw_ph(env, rc)) return 0;
  if (statsArr) {
    const jlong v[2] = {st.num_docs_scanned, st.num_entries_scanned_in_filter};
    (*env)->SetLongArrayRegion(env, statsArr, 0, 2, v);
  }
  return st.num_docs_scanned;
}

JNIEXPORT jlong JNICALL FN(resultNumGroups)(JNIEnv* env, jclass c, jlong res) { return ph_result_num_groups(PTR(res)); }

JNIEXPORT jint JNICALL FN(resultKeyType)(JNIEnv* env, jclass c, jlong res, jint g) { return ph_result_key_type(PTR(res), g); }

JNIEXPORT jint JNICALL FN(resultKeyEntrySize)(JNIEnv* env, jclass c, jlong res, jint g) {
  return ph_result_key_entry_size(PTR(res), g);
}

/* zero-copy views of the result's pinned host columns, valid until resultDestroy */
JNIEXPORT jobject JNICALL FN(resultKeyBuffer)(JNIEnv* env, jclass c, jlong res, jint g) {
  const int64_t n = ph_result_num_groups(PTR(res));
  const int es = ph_result_key_entry_size(PTR(res), g);
  return (*env)->NewDirectByteBuffer(env, (void*)ph_result_key_data(PTR(res), g), (jlong)n * es);
}

JNIEXPORT jobject JNICALL FN(resultAggregationBuffer)(JNIEnv* env, jclass c, jlong res, jint a, jint entryBytes) {
  const int64_t n = ph_result_num_groups(PTR(res));
  return (*env)->NewDirectByteBuffer(env, (void*)ph_result_aggregation_data(PTR(res), a), (jlong)n * entryBytes);
}

/* ph_exec_stats: numDocsScanned, numEntriesScannedInFilter, numEntriesScannedPostFilter, numTotalDocs,
 * numSegmentsProcessed, numSegmentsMatched, numGroupsLimitReached */
JNIEXPORT void JNICALL FN(resultStats)(JNIEnv* env, jclass c, jlong res, jlongArray out) {
  ph_exec_stats st;
  if (throw_ph(env, ph_result_stats(PTR(res), &st))) return;
  const jlong v[7] = {st.num_docs_scanned, st.num_entries_scanned_in_filter, st.num_entries_scanned_post_filter,
                      st.num_total_docs, st.num_segments_processed, st.num_segments_matched,
                      st.num_groups_limit_reached};
  (*env)->SetLongArrayRegion(env, out, 0, 7, v);
}

JNIEXPORT void JNICALL FN(resultDestroy)(JNIEnv* env, jclass c, jlong res) { throw_ph(env, ph_result_destroy(PTR(res))); }
