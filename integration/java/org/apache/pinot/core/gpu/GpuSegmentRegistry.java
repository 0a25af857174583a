package org.apache.pinot.core.gpu;

import java.io.File;
import java.util.List;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.atomic.AtomicInteger;
import org.apache.pinot.segment.spi.IndexSegment;


/**
 * Device-resident segments of one GPU context: pinned from the segment's own directory with ph_segment_load_dir
 * (SegmentMetadata.getIndexDir(), v3 columns.psf or v1 files) when the server loads it, released when the segment is
 * destroyed (ImmutableSegmentImpl.destroy, ImmutableSegmentImpl.java:249).  A query runs on the GPU only when every
 * segment it touches is pinned (else the CPU plan).
 *
 * Entries are keyed by segment NAME (what a query's IndexSegment list resolves through) but carry the IndexSegment
 * they were pinned for: a refresh loads the new IndexSegment before the old one is destroyed, so the new copy replaces
 * the old entry (the old copy's bytes are released first when the budget is checked), and the old segment's destroy
 * hook then finds an entry that is not its own and leaves it alone.  The HBM budget is enforced per device
 * (ph_segment_device), since the library places each segment on one device of the context.
 *
 * A query holds its segments through a Lease (acquire): every entry is reference-counted -- one reference for the
 * registry, one per in-flight query -- and ph_segment_unpin runs when the LAST reference goes, so a refresh or a destroy
 * that removes an entry while a query still runs on its handle only drops the registry's reference (the query's
 * release then unpins).  A lease cannot be taken on an entry whose last reference is already gone.
 */
public final class GpuSegmentRegistry {
  private static final class Entry {
    final IndexSegment _segment;
    final long _handle;
    final long _bytes;
    final int _device;
    final AtomicInteger _refs = new AtomicInteger(1);  // the registry's own reference

    Entry(IndexSegment segment, long handle, long bytes, int device) {
      _segment = segment;
      _handle = handle;
      _bytes = bytes;
      _device = device;
    }

    boolean retain() {
      for (;;) {
        int r = _refs.get();
        if (r == 0) {
          return false;  // already released by its last holder: unpinned or about to be
        }
        if (_refs.compareAndSet(r, r + 1)) {
          return true;
        }
      }
    }

    void release() {
      if (_refs.decrementAndGet() == 0) {
        PinotHipJni.segmentUnpin(_handle);
      }
    }
  }

  /** The device handles of one query's segments, held until close() (idempotent). */
  public static final class Lease implements AutoCloseable {
    private final Entry[] _entries;
    private final long[] _handles;
    private boolean _closed;

    Lease(Entry[] entries) {
      _entries = entries;
      _handles = new long[entries.length];
      for (int i = 0; i < entries.length; i++) {
        _handles[i] = entries[i]._handle;
      }
    }

    public long[] handles() {
      return _handles;
    }

    @Override
    public synchronized void close() {
      if (_closed) {
        return;
      }
      _closed = true;
      for (Entry e : _entries) {
        e.release();
      }
    }
  }

  private final long _ctx;
  private final long _hbmBudgetPerDevice;  // bytes the pinned segments may hold on each device of the context
  private final ConcurrentHashMap<String, Entry> _pinned = new ConcurrentHashMap<>();
  private final long[] _held;  // pinned bytes per device index, guarded by `this`

  public GpuSegmentRegistry(long ctx, long hbmBudgetPerDevice, int numDevices) {
    _ctx = ctx;
    _hbmBudgetPerDevice = hbmBudgetPerDevice;
    _held = new long[Math.max(1, numDevices)];
  }

  /** Hook for ImmutableSegmentLoader.load (after the CPU load succeeded). */
  public void onSegmentLoaded(IndexSegment segment) {
    File dir = segment.getSegmentMetadata().getIndexDir();
    if (dir == null) {
      return;  // mutable / consuming segments stay on the CPU path
    }
    String name = segment.getSegmentName();
    long handle;
    try {
      handle = PinotHipJni.segmentLoadDir(_ctx, dir.getAbsolutePath(), null);
    } catch (RuntimeException e) {
      // unsupported layout (raw / multi-value columns only, legacy padding, a packed stream past 2 GiB, out of HBM):
      // CPU path for this segment -- and never the GPU copy of an older version of it
      dropStale(name, segment);
      return;
    }
    // admission: the segment stays pinned only while the pinned segments of its device fit that device's budget
    // (measured footprint, ph_segment_device_bytes: columns plus the streams derived at pin); a refreshed segment's
    // old copy on the same device does not count against its replacement
    long bytes = PinotHipJni.segmentDeviceBytes(handle);
    int device = Math.max(0, Math.min(_held.length - 1, PinotHipJni.segmentDevice(handle)));
    Entry old;
    boolean admitted;
    synchronized (this) {
      old = _pinned.get(name);
      long oldOnDevice = old != null && old._device == device ? old._bytes : 0;
      if (_held[device] - oldOnDevice + bytes > _hbmBudgetPerDevice) {
        old = _pinned.remove(name);  // the refreshed data is not on the GPU: the old copy must not serve queries
        if (old != null) {
          _held[old._device] -= old._bytes;
        }
        admitted = false;
      } else {
        _pinned.put(name, new Entry(segment, handle, bytes, device));
        _held[device] += bytes;
        if (old != null) {
          _held[old._device] -= old._bytes;
        }
        admitted = true;
      }
    }
    if (!admitted) {
      PinotHipJni.segmentUnpin(handle);  // over the device's budget: CPU path (never visible to a query)
    }
    if (old != null) {
      old.release();  // segment refresh: the new copy (or the CPU path) replaces the old one once its queries finish
    }
  }

  /** Hook for ImmutableSegmentImpl.destroy: releases the entry only if it belongs to this IndexSegment. */
  public void onSegmentDestroyed(IndexSegment segment) {
    Entry e;
    synchronized (this) {
      e = _pinned.get(segment.getSegmentName());
      if (e == null || e._segment != segment) {
        return;  // already replaced by a refreshed copy (or never pinned)
      }
      _pinned.remove(segment.getSegmentName());
      _held[e._device] -= e._bytes;
    }
    e.release();  // unpinned now, or by the last query still holding it
  }

  private void dropStale(String name, IndexSegment replacement) {
    Entry old;
    synchronized (this) {
      old = _pinned.get(name);
      if (old == null || old._segment == replacement) {
        return;
      }
      _pinned.remove(name);
      _held[old._device] -= old._bytes;
    }
    old.release();
  }

  /**
   * A lease on the device handles of the query's segments, or null when one of them is not pinned (as this very
   * IndexSegment).  The caller closes it when its device calls are done.
   */
  public Lease acquire(List<IndexSegment> segments) {
    Entry[] out = new Entry[segments.size()];
    for (int i = 0; i < out.length; i++) {
      IndexSegment s = segments.get(i);
      Entry e = _pinned.get(s.getSegmentName());
      if (e == null || e._segment != s || !e.retain()) {
        for (int j = 0; j < i; j++) {
          out[j].release();
        }
        return null;
      }
      out[i] = e;
    }
    return new Lease(out);
  }
}
