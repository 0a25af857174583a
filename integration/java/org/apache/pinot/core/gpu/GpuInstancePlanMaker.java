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
  public static final String GPU_DEVICE_KEY = "pinot.server.query.executor.gpu.device";
  private long _ctx;
  private GpuSegmentRegistry _segments;

  @Override
  public void init(PinotConfiguration queryExecutorConfig) {
    super.init(queryExecutorConfig);
    _ctx = PinotHipJni.ctxCreate(queryExecutorConfig.getProperty(GPU_DEVICE_KEY, 0));
    _segments = new GpuSegmentRegistry(_ctx);
  }

  public GpuSegmentRegistry segments() {
    return _segments;
  }

  @Override
  public Plan makeInstancePlan(List<IndexSegment> indexSegments, QueryContext queryContext,
      ExecutorService executorService, ServerMetrics serverMetrics) {
    // the stock per-segment plan nodes: building them applies the query options (numGroupsLimit, trim sizes,
    // InstancePlanMakerImplV2.applyQueryOptions :166-229, called from makeSegmentPlanNode :254) and they are the
    // CPU fallback if the library declines the query at execution time
    List<PlanNode> segmentPlans = new ArrayList<>(indexSegments.size());
    for (IndexSegment segment : indexSegments) {
      segmentPlans.add(makeSegmentPlanNode(segment, queryContext));
    }
    GpuQuery q = GpuQuery.compile(queryContext);
    long[] handles = q == null ? null : _segments.handles(indexSegments);
    if (handles == null) {
      return super.makeInstancePlan(indexSegments, queryContext, executorService, serverMetrics);
    }
    GpuCombinePlanNode combine = new GpuCombinePlanNode(_ctx, q, handles, segmentPlans, queryContext, executorService);
    return new GlobalPlanImplV0(
        new InstanceResponsePlanNode(combine, indexSegments, Collections.emptyList(), queryContext));
  }
}
