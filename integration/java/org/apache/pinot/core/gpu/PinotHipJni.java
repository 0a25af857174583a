package org.apache.pinot.core.gpu;

import java.nio.ByteBuffer;

/**
 * JNI declarations of libpinot_hip.so (include/pinot_hip.h) through the shim integration/jni/pinot_hip_jni.c.
 * Handles are native pointers carried as longs.  JNI is the portable binding for the JDKs the reference supports
 * (release 11, pom.xml:112); an FFM binding over the same C-ABI is possible on JDK >= 22 (INTEGRATION.md).
 */
public final class PinotHipJni {
  static {
    System.loadLibrary("pinot_hip_jni");  // links libpinot_hip.so
  }

  private PinotHipJni() {
  }

  // ph_data_type / ph_aggregation_type / ph_filter_type / ph_predicate_type / ph_expr_op
  public static final int INT = 0, LONG = 1, FLOAT = 2, DOUBLE = 3, STRING = 4;
  public static final int AGG_COUNT = 0, AGG_SUM = 1, AGG_MIN = 2, AGG_MAX = 3, AGG_DISTINCTCOUNTHLL = 4;
  public static final int FILTER_AND = 0, FILTER_OR = 1, FILTER_NOT = 2, FILTER_PREDICATE = 3;
  public static final int PRED_EQ = 0, PRED_NOT_EQ = 1, PRED_IN = 2, PRED_NOT_IN = 3, PRED_RANGE = 4;
  public static final int EXPR_NONE = 0, EXPR_MULT = 1, EXPR_SUB = 2, EXPR_ADD = 3;

  static native long ctxCreate(int device);                                              // ph_ctx_create
  static native long ctxCreateMulti(int[] devices);                                      // ph_ctx_create_multi
  static native void ctxDestroy(long ctx);                                               // ph_ctx_destroy

  static native long segmentLoadDir(long ctx, String segmentDir, String[] columns);      // ph_segment_load_dir
  static native void segmentUnpin(long segment);                                         // ph_segment_unpin
  static native long segmentDeviceBytes(long segment);                                   // ph_segment_device_bytes
  static native int segmentDevice(long segment);                                         // ph_segment_device

  static native void tableSetDictionary(long ctx, String column, int dataType, ByteBuffer sortedValues, long count,
      int entrySize);                                                                    // ph_table_set_dictionary
  static native void tableSetColumnType(long ctx, String column, int dataType);          // ph_table_set_column_type

  /** ph_query_execute; descriptor layout in pinot_hip_jni.c (GpuQuery builds it). */
  static native long queryExecute(long ctx, int[] descriptor, String[] strings, long numGroupsLimit, long endTimeMs,
      long[] segments);

  /**
   * ph_filter_execute over one segment (GpuFilterOperator): the WHERE clause of `descriptor` (GpuQuery.compileFilter);
   * docWords (ceil(numDocs / 64) longs, bit i of word w = doc 64 w + i) receives the doc set, or null for the count
   * alone; statsOut[0] = matching docs, statsOut[1] = numEntriesScannedInFilter.  Returns the matching docs.
   */
  static native long filterExecute(long ctx, int[] descriptor, String[] strings, long endTimeMs, long segment,
      long[] docWords, long[] statsOut);

  static native long resultNumGroups(long result);                                       // ph_result_num_groups
  static native int resultKeyType(long result, int groupByIndex);                        // ph_result_key_type
  static native int resultKeyEntrySize(long result, int groupByIndex);                   // ph_result_key_entry_size
  static native ByteBuffer resultKeyBuffer(long result, int groupByIndex);               // ph_result_key_data
  static native ByteBuffer resultAggregationBuffer(long result, int aggIndex, int entryBytes);
  static native void resultStats(long result, long[] out7);                              // ph_result_stats
  static native void resultDestroy(long result);                                         // ph_result_destroy
}
