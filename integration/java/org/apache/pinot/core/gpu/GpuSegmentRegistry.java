package org.apache.pinot.core.gpu;

import java.io.File;
import java.util.List;
import java.util.concurrent.ConcurrentHashMap;
import org.apache.pinot.segment.spi.IndexSegment;


/**
 * Device-resident segments of one GPU: pinned from the segment's own directory with ph_segment_load_dir
 * (SegmentMetadata.getIndexDir(), v3 columns.psf or v1 files) when the server loads it, released when the segment is
 * destroyed (ImmutableSegmentImpl.destroy, ImmutableSegmentImpl.java:249).  A query runs on the GPU only when every
 * segment it touches is pinned (else the CPU plan).
 */
public final class GpuSegmentRegistry {
  private final long _ctx;
  private final ConcurrentHashMap<String, Long> _pinned = new ConcurrentHashMap<>();

  public GpuSegmentRegistry(long ctx) {
    _ctx = ctx;
  }

  /** Hook for ImmutableSegmentLoader.load (after the CPU load succeeded). */
  public void onSegmentLoaded(IndexSegment segment) {
    File dir = segment.getSegmentMetadata().getIndexDir();
    if (dir == null) {
      return;  // mutable / consuming segments stay on the CPU path
    }
    try {
      long handle = PinotHipJni.segmentLoadDir(_ctx, dir.getAbsolutePath(), null);
      Long old = _pinned.put(segment.getSegmentName(), handle);
      if (old != null) {
        PinotHipJni.segmentUnpin(old);  // segment refresh: the new copy replaces the old one
      }
    } catch (RuntimeException e) {
      // unsupported layout (raw / multi-value columns only, legacy padding, out of HBM): CPU path for this segment
    }
  }

  /** Hook for ImmutableSegmentImpl.destroy. */
  public void onSegmentDestroyed(String segmentName) {
    Long handle = _pinned.remove(segmentName);
    if (handle != null) {
      PinotHipJni.segmentUnpin(handle);
    }
  }

  /** Device handles of the query's segments, or null when one of them is not pinned. */
  public long[] handles(List<IndexSegment> segments) {
    long[] out = new long[segments.size()];
    for (int i = 0; i < out.length; i++) {
      Long h = _pinned.get(segments.get(i).getSegmentName());
      if (h == null) {
        return null;
      }
      out[i] = h;
    }
    return out;
  }
}
