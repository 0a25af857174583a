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

#define FN(name) Java_org_apache_pinot_core_gpu_PinotHipJni_##name
#define PTR(x) ((void*)(intptr_t)(x))

JNIEXPORT jlong JNICALL FN(ctxCreate)(JNIEnv* env, jclass c, jint device) {
  ph_ctx* ctx = NULL;
  throw_ph(env, ph_ctx_create(device, &ctx));
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL FN(ctxDestroy)(JNIEnv* env, jclass c, jlong ctx) { throw_ph(env, ph_ctx_destroy(PTR(ctx))); }

/* ImmutableSegmentLoader.load -> pin the segment's directory (ph_segment_load_dir); columns == null: all */
JNIEXPORT jlong JNICALL FN(segmentLoadDir)(JNIEnv* env, jclass c, jlong ctx, jstring dir, jobjectArray columns) {
  const char* d = (*env)->GetStringUTFChars(env, dir, NULL);
  const jsize n = columns ? (*env)->GetArrayLength(env, columns) : 0;
  const char** cols = n ? (const char**)calloc((size_t)n, sizeof(char*)) : NULL;
  for (jsize i = 0; i < n; ++i)
    cols[i] = (*env)->GetStringUTFChars(env, (jstring)(*env)->GetObjectArrayElement(env, columns, i), NULL);
  ph_segment* seg = NULL;
  const int rc = ph_segment_load_dir(PTR(ctx), d, cols, (int32_t)n, &seg);
  for (jsize i = 0; i < n; ++i)
    (*env)->ReleaseStringUTFChars(env, (jstring)(*env)->GetObjectArrayElement(env, columns, i), cols[i]);
  free(cols);
  (*env)->ReleaseStringUTFChars(env, dir, d);
  throw_ph(env, rc);
  return (jlong)(intptr_t)seg;
}

JNIEXPORT void JNICALL FN(segmentUnpin)(JNIEnv* env, jclass c, jlong seg) { throw_ph(env, ph_segment_unpin(PTR(seg))); }

JNIEXPORT jlong JNICALL FN(segmentDeviceBytes)(JNIEnv* env, jclass c, jlong seg) {
  return ph_segment_device_bytes(PTR(seg));
}

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
 *    per aggregation: type, column, log2m, column2, exprOp]                                                      */
JNIEXPORT jlong JNICALL FN(queryExecute)(JNIEnv* env, jclass c, jlong ctx, jintArray descArr, jobjectArray strArr,
                                         jlong numGroupsLimit, jlong endTimeMs, jlongArray segArr) {
  const jsize nd = (*env)->GetArrayLength(env, descArr), ns = (*env)->GetArrayLength(env, strArr);
  jint* desc = (*env)->GetIntArrayElements(env, descArr, NULL);
  const char** strs = (const char**)calloc((size_t)(ns ? ns : 1), sizeof(char*));
  for (jsize i = 0; i < ns; ++i)
    strs[i] = (*env)->GetStringUTFChars(env, (jstring)(*env)->GetObjectArrayElement(env, strArr, i), NULL);
#define S(i) ((i) >= 0 && (i) < ns ? strs[(i)] : NULL)
  int k = 0;
  ph_query q;
  memset(&q, 0, sizeof q);
  q.num_filter_nodes = desc[k++];
  q.filter_root = desc[k++];
  q.num_predicates = desc[k++];
  q.num_group_by = desc[k++];
  q.num_aggregations = desc[k++];
  ph_filter_node* nodes = (ph_filter_node*)calloc((size_t)q.num_filter_nodes + 1, sizeof(ph_filter_node));
  ph_predicate* preds = (ph_predicate*)calloc((size_t)q.num_predicates + 1, sizeof(ph_predicate));
  const char** gby = (const char**)calloc((size_t)q.num_group_by + 1, sizeof(char*));
  ph_aggregation* aggs = (ph_aggregation*)calloc((size_t)q.num_aggregations + 1, sizeof(ph_aggregation));
  int32_t* ints = (int32_t*)calloc((size_t)nd + 1, sizeof(int32_t));  /* children lists live here */
  const char** vals = (const char**)calloc((size_t)nd + 1, sizeof(char*));
  int ki = 0, kv = 0;
  for (int i = 0; i < q.num_filter_nodes; ++i) {
    nodes[i].type = desc[k++];
    nodes[i].num_children = desc[k++];
    nodes[i].predicate = desc[k++];
    nodes[i].children = ints + ki;
    for (int j = 0; j < nodes[i].num_children; ++j) ints[ki++] = desc[k++];
  }
  for (int i = 0; i < q.num_predicates; ++i) {
    preds[i].type = desc[k++];
    preds[i].column = S(desc[k]); k++;
    preds[i].num_values = desc[k++];
    preds[i].values = vals + kv;
    for (int j = 0; j < preds[i].num_values; ++j) vals[kv++] = S(desc[k++]);
    preds[i].lower = S(desc[k]); k++;
    preds[i].upper = S(desc[k]); k++;
    preds[i].lower_inclusive = desc[k++];
    preds[i].upper_inclusive = desc[k++];
  }
  for (int i = 0; i < q.num_group_by; ++i) gby[i] = S(desc[k++]);
  for (int i = 0; i < q.num_aggregations; ++i) {
    aggs[i].type = desc[k++];
    aggs[i].column = S(desc[k]); k++;
    aggs[i].log2m = desc[k++];
    aggs[i].column2 = S(desc[k]); k++;
    aggs[i].expr_op = desc[k++];
  }
  q.filter_nodes = nodes;
  q.predicates = preds;
  q.group_by = gby;
  q.aggregations = aggs;
  q.num_groups_limit = numGroupsLimit;
  q.end_time_ms = endTimeMs;
  const jsize nseg = (*env)->GetArrayLength(env, segArr);
  jlong* segs = (*env)->GetLongArrayElements(env, segArr, NULL);
  ph_segment** sp = (ph_segment**)calloc((size_t)(nseg ? nseg : 1), sizeof(ph_segment*));
  for (jsize i = 0; i < nseg; ++i) sp[i] = (ph_segment*)PTR(segs[i]);
  ph_result* res = NULL;
  const int rc = ph_query_execute(PTR(ctx), &q, sp, (int32_t)nseg, &res);
  free(sp);
  (*env)->ReleaseLongArrayElements(env, segArr, segs, JNI_ABORT);
  free(nodes); free(preds); free(gby); free(aggs); free(ints); free(vals);
  for (jsize i = 0; i < ns; ++i)
    (*env)->ReleaseStringUTFChars(env, (jstring)(*env)->GetObjectArrayElement(env, strArr, i), strs[i]);
  free(strs);
  (*env)->ReleaseIntArrayElements(env, descArr, desc, JNI_ABORT);
#undef S
  throw_ph(env, rc);
  return (jlong)(intptr_t)res;
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
