package org.apache.pinot.core.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;
import java.util.Collections;
import java.util.Iterator;
import java.util.List;
import java.util.NoSuchElementException;
import java.util.Set;
import com.clearspring.analytics.stream.cardinality.HyperLogLog;
import com.clearspring.analytics.stream.cardinality.RegisterSet;
import org.apache.pinot.common.request.context.ExpressionContext;
import org.apache.pinot.common.utils.DataSchema;
import org.apache.pinot.core.common.Operator;
import org.apache.pinot.core.operator.BaseOperator;
import org.apache.pinot.core.operator.BaseProjectOperator;
import org.apache.pinot.core.operator.ExecutionStatistics;
import org.apache.pinot.core.operator.blocks.results.AggregationResultsBlock;
import org.apache.pinot.core.operator.blocks.results.BaseResultsBlock;
import org.apache.pinot.core.operator.blocks.results.GroupByResultsBlock;
import org.apache.pinot.core.operator.blocks.ValueBlock;
import org.apache.pinot.core.operator.query.AggregationOperator;
import org.apache.pinot.core.operator.query.FastFilteredCountOperator;
import org.apache.pinot.core.operator.query.GroupByOperator;
import org.apache.pinot.core.operator.query.SelectionOnlyOperator;
import org.apache.pinot.core.plan.DocIdSetPlanNode;
import org.apache.pinot.core.plan.PlanNode;
import org.apache.pinot.core.plan.ProjectPlanNode;
import org.apache.pinot.core.query.aggregation.function.AggregationFunction;
import org.apache.pinot.core.query.aggregation.function.AggregationFunctionUtils;
import org.apache.pinot.core.query.aggregation.function.DistinctCountHLLAggregationFunction;
import org.apache.pinot.core.query.aggregation.groupby.AggregationGroupByResult;
import org.apache.pinot.core.query.aggregation.groupby.DoubleGroupByResultHolder;
import org.apache.pinot.core.query.aggregation.groupby.GroupByResultHolder;
import org.apache.pinot.core.query.aggregation.groupby.GroupKeyGenerator;
import org.apache.pinot.core.query.aggregation.groupby.ObjectGroupByResultHolder;
import org.apache.pinot.core.query.request.context.QueryContext;
import org.apache.pinot.core.query.request.context.utils.QueryContextUtils;
import org.apache.pinot.core.query.selection.SelectionOperatorUtils;
import org.apache.pinot.segment.spi.AggregationFunctionType;
import org.apache.pinot.segment.spi.IndexSegment;


/**
 * Segment-level GPU plan (SURVEY 8(b) plug point 2; PlanMaker.makeSegmentPlanNode, InstancePlanMakerImplV2.java:232-249):
 * the per-segment plan node of a pinned segment, whose operators the stock combine (GroupByCombineOperator /
 * AggregationCombineOperator / SelectionOnlyCombineOperator) merges unchanged.
 *
 *  - whole query on the GPU (GpuQuery.compile accepts it): ph_query_execute over this ONE segment; a group-by returns
 *    GroupByResultsBlock(DataSchema, AggregationGroupByResult, ctx) (GroupByResultsBlock.java:62) whose
 *    GroupKeyGenerator / GroupByResultHolders are views of the result columns, an aggregation
 *    AggregationResultsBlock(functions, results, ctx) (AggregationResultsBlock.java:50);
 *  - otherwise the GPU evaluates the WHERE clause (GpuFilterOperator over ph_filter_execute) and the reference's
 *    operators run above it exactly as GroupByPlanNode (:72-108), AggregationPlanNode (:95-150) and
 *    SelectionPlanNode (:54-73) wire them: FastFilteredCountOperator for COUNT(*), ProjectPlanNode(..., filterOperator)
 *    under GroupByOperator / AggregationOperator / SelectionOnlyOperator;
 *  - any other shape: the stock plan node.
 */
public class GpuSegmentPlanNode implements PlanNode {
  private final long _ctx;
  private final GpuSegmentRegistry _registry;
  private final IndexSegment _segment;
  private final QueryContext _queryContext;
  private final PlanNode _stock;

  public GpuSegmentPlanNode(long ctx, GpuSegmentRegistry registry, IndexSegment segment, QueryContext queryContext,
      PlanNode stock) {
    _ctx = ctx;
    _registry = registry;
    _segment = segment;
    _queryContext = queryContext;
    _stock = stock;
  }

  @Override
  public Operator<?> run() {
    QueryContext ctx = _queryContext;
    if (ctx.isNullHandlingEnabled() || ctx.hasFilteredAggregations()) {
      return _stock.run();
    }
    int numTotalDocs = _segment.getSegmentMetadata().getTotalDocs();
    if (QueryContextUtils.isAggregationQuery(ctx)) {
      GpuQuery whole = GpuQuery.compile(ctx);
      GpuSegmentRegistry.Lease lease = _registry.acquire(Collections.singletonList(_segment));
      if (lease == null) {
        return _stock.run();
      }
      if (whole != null) {
        return new GpuSegmentOperator(whole, lease);
      }
      GpuFilterOperator filter = filterOperator(lease, numTotalDocs);
      if (filter == null) {
        lease.close();
        return _stock.run();
      }
      AggregationFunction[] functions = ctx.getAggregationFunctions();
      List<ExpressionContext> groupBy = ctx.getGroupByExpressions();
      if (groupBy != null) {
        Set<ExpressionContext> expressions = AggregationFunctionUtils.collectExpressionsToTransform(functions, groupBy);
        BaseProjectOperator<?> project = new ProjectPlanNode(_segment, ctx, expressions,
            DocIdSetPlanNode.MAX_DOC_PER_CALL, filter).run();
        return new GroupByOperator(ctx, groupBy.toArray(new ExpressionContext[0]), project, numTotalDocs, false);
      }
      if (functions.length == 1 && functions[0].getType() == AggregationFunctionType.COUNT) {
        return new FastFilteredCountOperator(ctx, filter, _segment.getSegmentMetadata());  // canOptimizeCount
      }
      Set<ExpressionContext> expressions = AggregationFunctionUtils.collectExpressionsToTransform(functions, null);
      BaseProjectOperator<?> project = new ProjectPlanNode(_segment, ctx, expressions,
          DocIdSetPlanNode.MAX_DOC_PER_CALL, filter).run();
      return new AggregationOperator(ctx, project, numTotalDocs, false);
    }
    if (QueryContextUtils.isSelectionQuery(ctx) && ctx.getOrderByExpressions() == null && ctx.getLimit() > 0) {
      GpuSegmentRegistry.Lease lease = _registry.acquire(Collections.singletonList(_segment));
      if (lease == null) {
        return _stock.run();
      }
      GpuFilterOperator filter = filterOperator(lease, numTotalDocs);
      if (filter == null) {
        lease.close();
        return _stock.run();
      }
      List<ExpressionContext> expressions = SelectionOperatorUtils.extractExpressions(ctx, _segment);
      int maxDocsPerCall = Math.min(ctx.getLimit(), DocIdSetPlanNode.MAX_DOC_PER_CALL);
      BaseProjectOperator<?> project = new ProjectPlanNode(_segment, ctx, expressions, maxDocsPerCall, filter).run();
      return new SelectionOnlyOperator(_segment, ctx, expressions, project);
    }
    return _stock.run();
  }

  // the WHERE clause on the GPU, or null (no filter -- the stock MatchAll plan is as cheap -- or a predicate shape the
  // library does not take)
  private GpuFilterOperator filterOperator(GpuSegmentRegistry.Lease lease, int numTotalDocs) {
    if (_queryContext.getFilter() == null) {
      return null;
    }
    GpuQuery filter = GpuQuery.compileFilter(_queryContext.getFilter(), _queryContext.getEndTimeMs());
    return filter == null ? null : new GpuFilterOperator(_ctx, filter, lease, numTotalDocs);
  }

  /**
   * The whole per-segment query as one ph_query_execute over this segment (what GroupByOperator / AggregationOperator
   * return for it).  PH_ERR_UNSUPPORTED at execution runs the stock operator instead.
   */
  private final class GpuSegmentOperator extends BaseOperator<BaseResultsBlock> {
    private static final String EXPLAIN_NAME = "SEGMENT_GPU";
    private final GpuQuery _query;
    private final GpuSegmentRegistry.Lease _lease;
    private final long[] _stats = new long[7];
    private Operator<?> _fallback;

    GpuSegmentOperator(GpuQuery query, GpuSegmentRegistry.Lease lease) {
      _query = query;
      _lease = lease;
    }

    @Override
    protected BaseResultsBlock getNextBlock() {
      long res;
      try {
        res = PinotHipJni.queryExecute(_ctx, _query._descriptor, _query._strings, _query._numGroupsLimit,
            _query._endTimeMs, _lease.handles());
      } catch (UnsupportedOperationException e) {
        _fallback = _stock.run();
        return (BaseResultsBlock) _fallback.nextBlock();
      } finally {
        _lease.close();
      }
      try {
        PinotHipJni.resultStats(res, _stats);
        return _queryContext.getGroupByExpressions() == null ? aggregation(res) : groupBy(res);
      } finally {
        PinotHipJni.resultDestroy(res);
      }
    }

    private BaseResultsBlock aggregation(long res) {
      AggregationFunction[] functions = _queryContext.getAggregationFunctions();
      List<Object> results = new java.util.ArrayList<>(functions.length);
      for (int k = 0; k < functions.length; k++) {
        results.add(intermediate(functions[k], column(res, k, functions[k]), 0));
      }
      return new AggregationResultsBlock(functions, results, _queryContext);
    }

    // GroupByResultsBlock(DataSchema, AggregationGroupByResult, ctx): the group keys as a GroupKeyGenerator over the
    // result rows, each function's results in the holder its extractGroupByResult reads (Double holders for COUNT /
    // SUM / MIN / MAX, HyperLogLog objects for DISTINCTCOUNTHLL); GroupByCombineOperator.processSegments (:161-176)
    // iterates exactly that
    private BaseResultsBlock groupBy(long res) {
      List<ExpressionContext> groupBy = _queryContext.getGroupByExpressions();
      AggregationFunction[] functions = _queryContext.getAggregationFunctions();
      int nk = groupBy.size();
      int n = (int) PinotHipJni.resultNumGroups(res);
      Object[][] keys = new Object[n][nk];
      for (int g = 0; g < nk; g++) {
        int type = PinotHipJni.resultKeyType(res, g);
        int size = PinotHipJni.resultKeyEntrySize(res, g);
        ByteBuffer b = PinotHipJni.resultKeyBuffer(res, g).order(ByteOrder.nativeOrder());
        for (int r = 0; r < n; r++) {
          keys[r][g] = keyValue(b, type, size, r);
        }
      }
      GroupByResultHolder[] holders = new GroupByResultHolder[functions.length];
      for (int k = 0; k < functions.length; k++) {
        ByteBuffer col = column(res, k, functions[k]);
        if (functions[k].getType() == AggregationFunctionType.DISTINCTCOUNTHLL) {
          ObjectGroupByResultHolder h = new ObjectGroupByResultHolder(n, n);
          for (int r = 0; r < n; r++) {
            h.setValueForKey(r, intermediate(functions[k], col, r));
          }
          holders[k] = h;
        } else {
          DoubleGroupByResultHolder h = new DoubleGroupByResultHolder(n, n, 0.0);
          for (int r = 0; r < n; r++) {
            Object v = intermediate(functions[k], col, r);
            h.setValueForKey(r, v instanceof Long ? (double) (Long) v : (Double) v);
          }
          holders[k] = h;
        }
      }
      DataSchema schema = GpuResultSchema.of(_queryContext, res);
      GroupByResultsBlock block = new GroupByResultsBlock(schema,
          new AggregationGroupByResult(new RowKeys(keys), functions, holders), _queryContext);
      block.setNumGroupsLimitReached(_stats[6] != 0);
      return block;
    }

    @Override
    public ExecutionStatistics getExecutionStatistics() {
      if (_fallback != null) {
        return _fallback.getExecutionStatistics();
      }
      return new ExecutionStatistics(_stats[0], _stats[1], _stats[2], _stats[3]);
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
  }

  static Object keyValue(ByteBuffer b, int type, int size, int r) {
    switch (type) {
      case PinotHipJni.INT: return b.getInt(4 * r);
      case PinotHipJni.LONG: return b.getLong(8 * r);
      case PinotHipJni.FLOAT: return b.getFloat(4 * r);
      case PinotHipJni.DOUBLE: return b.getDouble(8 * r);
      default: {
        byte[] s = new byte[size];
        for (int i = 0; i < size; i++) {
          s[i] = b.get(r * size + i);
        }
        int len = 0;
        while (len < s.length && s[len] != 0) {
          len++;
        }
        return new String(s, 0, len, StandardCharsets.UTF_8);
      }
    }
  }

  static ByteBuffer column(long res, int k, AggregationFunction f) {
    int bytes = f.getType() == AggregationFunctionType.DISTINCTCOUNTHLL
        ? 1 << ((DistinctCountHLLAggregationFunction) f).getLog2m() : 8;
    return PinotHipJni.resultAggregationBuffer(res, k, bytes).order(ByteOrder.nativeOrder());
  }

  // intermediate results as the CPU functions produce them: COUNT Long, SUM / MIN / MAX Double, HLL HyperLogLog
  static Object intermediate(AggregationFunction f, ByteBuffer col, int row) {
    AggregationFunctionType t = f.getType();
    if (t == AggregationFunctionType.COUNT) {
      return col.getLong(8 * row);
    }
    if (t == AggregationFunctionType.DISTINCTCOUNTHLL) {
      int log2m = ((DistinctCountHLLAggregationFunction) f).getLog2m();
      int m = 1 << log2m;
      RegisterSet registers = new RegisterSet(m);
      for (int j = 0; j < m; j++) {
        registers.set(j, col.get(row * m + j) & 0xff);
      }
      return new HyperLogLog(log2m, registers);
    }
    return col.getDouble(8 * row);
  }

  /** GroupKeyGenerator over materialised result rows: group id = row (GroupKeyGenerator.java:28-84). */
  static final class RowKeys implements GroupKeyGenerator {
    private final Object[][] _keys;

    RowKeys(Object[][] keys) {
      _keys = keys;
    }

    @Override
    public int getGlobalGroupKeyUpperBound() {
      return _keys.length;
    }

    @Override
    public void generateKeysForBlock(ValueBlock valueBlock, int[] groupKeys) {
      throw new UnsupportedOperationException("keys come from the GPU result");
    }

    @Override
    public void generateKeysForBlock(ValueBlock valueBlock, int[][] groupKeys) {
      throw new UnsupportedOperationException("keys come from the GPU result");
    }

    @Override
    public int getCurrentGroupKeyUpperBound() {
      return _keys.length;
    }

    @Override
    public Iterator<GroupKey> getGroupKeys() {
      return new Iterator<GroupKey>() {
        private int _next;
        private final GroupKey _key = new GroupKey();

        @Override
        public boolean hasNext() {
          return _next < _keys.length;
        }

        @Override
        public GroupKey next() {
          if (_next >= _keys.length) {
            throw new NoSuchElementException();
          }
          _key._groupId = _next;
          _key._keys = _keys[_next++];
          return _key;
        }
      };
    }

    @Override
    public int getNumKeys() {
      return _keys.length;
    }
  }
}
