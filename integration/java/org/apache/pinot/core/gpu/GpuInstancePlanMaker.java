package org.apache.pinot.core.gpu;

import java.util.ArrayList;
import java.util.Collections;
import java.util.List;
import java.util.concurrent.ExecutorService;
import org.apache.pinot.common.metrics.ServerMetrics;
import org.apache.pinot.core.plan.GlobalPlanImplV0;
import org.apache.pinot.core.plan.InstanceResponsePlanNode;
import org.apache.pinot.core.plan.Plan;
import org.apache.pinot.core.plan.PlanNode;
import org.apache.pinot.core.plan.maker.InstancePlanMakerImplV2;
import org.apache.pinot.core.query.request.context.QueryContext;
import org.apache.pinot.segment.spi.IndexSegment;
import org.apache.pinot.spi.env.PinotConfiguration;


/**
 * The plug point (PlanMaker.java:37-67, selected by pinot.server.query.executor.plan.maker.class,
 * QueryExecutorConfig.java:31,50): aggregation / group-by queries whose shape GpuQuery accepts and whose segments are
 * all pinned run as ONE batched launch over every segment of the GPU, combine included (GpuCombinePlanNode); anything
 * else, and any PH_ERR_UNSUPPORTED at execution, takes the stock plan of InstancePlanMakerImplV2.
 */
public class GpuInstancePlanMaker extends InstancePlanMakerImplV2 {
  // next to the executor's own keys (CommonConstants.Server, pinot.server.query.executor.*)
  public static final String GPU_ENABLE_KEY = "pinot.server.query.executor.gpu.enable";
  /** Comma-separated HIP device ordinals the server's context spans (one ph_ctx over all of them). */
  public static final String GPU_DEVICES_KEY = "pinot.server.query.executor.gpu.devices";
  /** Single-device form (kept for compatibility): used when gpu.devices is absent. */
  public static final String GPU_DEVICE_KEY = "pinot.server.query.executor.gpu.device";
  /** HBM the pinned segments may hold per device, in bytes (default: 240 GB of a 288 GB MI355X). */
  public static final String GPU_HBM_BUDGET_KEY = "pinot.server.query.executor.gpu.hbm.budget";
  public static final long DEFAULT_HBM_BUDGET = 240L << 30;
  /**
   * "instance" (default): a query whose whole shape the library takes runs as ONE batched launch over all its
   * segments (GpuCombinePlanNode); "segment": every pinned segment gets its own GPU plan (GpuSegmentPlanNode) and the
   * stock combine merges them.  Either way, queries the instance plan does not take get the segment-level GPU plans
   * (their filters on the GPU, SURVEY 8(b) plug point 2).
   */
  public static final String GPU_MODE_KEY = "pinot.server.query.executor.gpu.mode";
  private long _ctx;
  private GpuSegmentRegistry _segments;
  private boolean _enabled;
  private boolean _instanceMode;

  @Override
  public void init(PinotConfiguration queryExecutorConfig) {
    super.init(queryExecutorConfig);
    _enabled = queryExecutorConfig.getProperty(GPU_ENABLE_KEY, true);
    _instanceMode = !"segment".equals(queryExecutorConfig.getProperty(GPU_MODE_KEY, "instance"));
    if (!_enabled) {
      return;  // the stock plan maker, unchanged
    }
    String devices = queryExecutorConfig.getProperty(GPU_DEVICES_KEY, "");
    int[] ords;
    if (devices.isEmpty()) {
      ords = new int[]{queryExecutorConfig.getProperty(GPU_DEVICE_KEY, 0)};
    } else {
      String[] parts = devices.split(",");
      ords = new int[parts.length];
      for (int i = 0; i < parts.length; i++) {
        ords[i] = Integer.parseInt(parts[i].trim());
      }
    }
    // one context over the device set: segments are placed by pinned rows and a query's per-device partials merge
    // inside the library (RCCL reduce-scatter over xGMI), as GroupByCombineOperator merges them in this JVM
    _ctx = ords.length == 1 ? PinotHipJni.ctxCreate(ords[0]) : PinotHipJni.ctxCreateMulti(ords);
    long budget = queryExecutorConfig.getProperty(GPU_HBM_BUDGET_KEY, DEFAULT_HBM_BUDGET);
    _segments = new GpuSegmentRegistry(_ctx, budget, ords.length);  // budget per device (ph_segment_device)
  }

  /** null when gpu.enable is false (the server's segment hooks then do nothing). */
  public GpuSegmentRegistry segments() {
    return _segments;
  }

  @Override
  public Plan makeInstancePlan(List<IndexSegment> indexSegments, QueryContext queryContext,
      ExecutorService executorService, ServerMetrics serverMetrics) {
    GpuQuery q = _enabled && _instanceMode ? GpuQuery.compile(queryContext) : null;
    GpuSegmentRegistry.Lease lease = q == null ? null : _segments.acquire(indexSegments);
    if (lease == null) {
      // the stock instance plan, whose per-segment nodes come from makeSegmentPlanNode below (GPU filters)
      return super.makeInstancePlan(indexSegments, queryContext, executorService, serverMetrics);
    }
    // the stock per-segment plan nodes: building them applies the query options (numGroupsLimit, trim sizes,
    // InstancePlanMakerImplV2.applyQueryOptions :166-229, called from makeSegmentPlanNode :254) and they are the
    // CPU fallback if the library declines the query at execution time
    List<PlanNode> segmentPlans = new ArrayList<>(indexSegments.size());
    for (IndexSegment segment : indexSegments) {
      segmentPlans.add(super.makeSegmentPlanNode(segment, queryContext));
    }
    GpuCombinePlanNode combine = new GpuCombinePlanNode(_ctx, q, lease, segmentPlans, queryContext, executorService);
    return new GlobalPlanImplV0(
        new InstanceResponsePlanNode(combine, indexSegments, Collections.emptyList(), queryContext));
  }

  /**
   * SURVEY 8(b) plug point 2 (PlanMaker.makeSegmentPlanNode, PlanMaker.java:53): the stock node (which applies the
   * per-segment query rewrites) wrapped in the GPU segment plan -- whole query on the GPU when GpuQuery takes it, else
   * the GPU filter under the reference's own operators; an unpinned segment keeps the stock node.
   */
  @Override
  public PlanNode makeSegmentPlanNode(IndexSegment indexSegment, QueryContext queryContext) {
    PlanNode stock = super.makeSegmentPlanNode(indexSegment, queryContext);
    if (!_enabled) {
      return stock;
    }
    return new GpuSegmentPlanNode(_ctx, _segments, indexSegment, queryContext, stock);
  }
}
