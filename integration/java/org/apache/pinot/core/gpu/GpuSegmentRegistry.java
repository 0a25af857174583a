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
  private final long _hbmBudget;  // bytes the pinned segments may hold over the context's devices
  private final ConcurrentHashMap<String, Long> _pinned = new ConcurrentHashMap<>();
  private final ConcurrentHashMap<String, Long> _bytes = new ConcurrentHashMap<>();
  private final java.util.concurrent.atomic.AtomicLong _held = new java.util.concurrent.atomic.AtomicLong();

  public GpuSegmentRegistry(long ctx, long hbmBudget) {
    _ctx = ctx;
    _hbmBudget = hbmBudget;
  }

  /** Hook for ImmutableSegmentLoader.load (after the CPU load succeeded). */
  public void onSegmentLoaded(IndexSegment segment) {
    File dir = segment.getSegmentMetadata().getIndexDir();
    if (dir == null) {
      return;  // mutable / consuming segments stay on the CPU path
    }
    try {
      long handle = PinotHipJni.segmentLoadDir(_ctx, dir.getAbsolutePath(), null);
      // admission: the segment stays pinned only while every pinned segment fits the HBM budget (its measured
      // footprint, ph_segment_device_bytes: columns plus the streams derived at pin); past it, the CPU path
      long bytes = PinotHipJni.segmentDeviceBytes(handle);
      if (_held.addAndGet(bytes) > _hbmBudget) {
        _held.addAndGet(-bytes);
        PinotHipJni.segmentUnpin(handle);
        return;
      }
      Long oldBytes = _bytes.put(segment.getSegmentName(), bytes);
      Long old = _pinned.put(segment.getSegmentName(), handle);
      if (old != null) {
        if (oldBytes != null) {
          _held.addAndGet(-oldBytes);
        }
        PinotHipJni.segmentUnpin(old);  // segment refresh: the new copy replaces the old one
      }
    } catch (RuntimeException e) {
      // unsupported layout (raw / multi-value columns only, legacy padding, a packed stream past 2 GiB, out of
      // HBM): CPU path for this segment
    }
  }

  /** Hook for ImmutableSegmentImpl.destroy. */
  public void onSegmentDestroyed(String segmentName) {
    Long handle = _pinned.remove(segmentName);
    if (handle != null) {
      Long bytes = _bytes.remove(segmentName);
      if (bytes != null) {
        _held.addAndGet(-bytes);
      }
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
