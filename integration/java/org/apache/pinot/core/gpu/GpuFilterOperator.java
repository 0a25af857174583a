package org.apache.pinot.core.gpu;

import java.util.Collections;
import java.util.List;
import org.apache.pinot.core.common.BlockDocIdSet;
import org.apache.pinot.core.common.Operator;
import org.apache.pinot.core.operator.dociditerators.BitmapDocIdIterator;
import org.apache.pinot.core.operator.filter.BaseFilterOperator;
import org.apache.pinot.core.operator.filter.BitmapCollection;
import org.roaringbitmap.BitSetUtil;
import org.roaringbitmap.buffer.ImmutableRoaringBitmap;
import org.roaringbitmap.buffer.MutableRoaringBitmap;


/**
 * The segment-level drop-in of SURVEY 8(b) plug point 2: what FilterPlanNode.run (FilterPlanNode.java:83-114) returns
 * for a segment pinned in HBM.  One ph_filter_execute evaluates the segment's whole WHERE clause on the GPU -- the same
 * leaf choice (sorted > inverted > range > scan) and predicate evaluators as the reference's operator tree -- and hands
 * back the matching docs as 64-bit words (bit i of word w = doc 64 w + i), the count and the tree's
 * numEntriesScannedInFilter.  Like BitmapBasedFilterOperator (BitmapBasedFilterOperator.java:29-82) it answers
 * getTrues() with a BitmapDocIdSet-shaped set, canOptimizeCount() / getNumMatchingDocs() (so AggregationPlanNode takes
 * FastFilteredCountOperator, :101-105) and getBitmaps(); everything above it -- projection, selection, the ~80 other
 * aggregation functions, distinct, filtered-aggregation siblings -- is the reference's own code over the GPU's doc set.
 *
 * The device call runs once, on the first getTrues / getNumMatchingDocs / getBitmaps, and releases the segment's
 * registry lease right after it (the handle cannot be unpinned while the call is in flight).
 */
public class GpuFilterOperator extends BaseFilterOperator {
  private static final String EXPLAIN_NAME = "FILTER_GPU";

  private final long _ctx;
  private final GpuQuery _filter;
  private final GpuSegmentRegistry.Lease _lease;  // one segment
  private MutableRoaringBitmap _docIds;
  private int _numMatchingDocs = -1;
  private long _numEntriesScannedInFilter;

  public GpuFilterOperator(long ctx, GpuQuery filter, GpuSegmentRegistry.Lease lease, int numDocs) {
    super(numDocs, false);
    _ctx = ctx;
    _filter = filter;
    _lease = lease;
  }

  private void evaluate() {
    if (_docIds != null) {
      return;
    }
    long[] words = new long[(_numDocs + 63) >>> 6];
    long[] stats = new long[2];  // numDocsScanned (matching docs), numEntriesScannedInFilter
    try {
      _numMatchingDocs = (int) PinotHipJni.filterExecute(_ctx, _filter._descriptor, _filter._strings,
          _filter._endTimeMs, _lease.handles()[0], words, stats);
    } finally {
      _lease.close();
    }
    _numEntriesScannedInFilter = stats[1];
    _docIds = BitSetUtil.bitmapOf(words).toMutableRoaringBitmap();  // the java.util.BitSet word layout
  }

  @Override
  protected BlockDocIdSet getTrues() {
    evaluate();
    return new GpuDocIdSet(_docIds, _numDocs, _numEntriesScannedInFilter);
  }

  @Override
  public boolean canOptimizeCount() {
    return true;
  }

  @Override
  public int getNumMatchingDocs() {
    evaluate();
    return _numMatchingDocs;
  }

  @Override
  public boolean canProduceBitmaps() {
    return true;
  }

  @Override
  public BitmapCollection getBitmaps() {
    evaluate();
    return new BitmapCollection(_numDocs, false, _docIds);
  }

  @Override
  @SuppressWarnings("rawtypes")
  public List<Operator> getChildOperators() {
    return Collections.emptyList();
  }

  @Override
  public String toExplainString() {
    return EXPLAIN_NAME;
  }

  /**
   * BitmapDocIdSet (BitmapDocIdSet.java:26-46) that reports the GPU-computed statistic of the filter tree it replaces
   * (BlockDocIdSet.getNumEntriesScannedInFilter: what the reference's scan iterators would have examined).
   */
  static final class GpuDocIdSet implements BlockDocIdSet {
    private final BitmapDocIdIterator _iterator;
    private final long _numEntriesScannedInFilter;

    GpuDocIdSet(ImmutableRoaringBitmap docIds, int numDocs, long numEntriesScannedInFilter) {
      _iterator = new BitmapDocIdIterator(docIds, numDocs);
      _numEntriesScannedInFilter = numEntriesScannedInFilter;
    }

    @Override
    public BitmapDocIdIterator iterator() {
      return _iterator;
    }

    @Override
    public long getNumEntriesScannedInFilter() {
      return _numEntriesScannedInFilter;
    }
  }
}
