package org.apache.pinot.core.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.Collections;
import java.util.List;
import java.util.concurrent.ExecutorService;
import com.clearspring.analytics.stream.cardinality.HyperLogLog;
import com.clearspring.analytics.stream.cardinality.RegisterSet;
import org.apache.pinot.common.request.context.ExpressionContext;
import org.apache.pinot.common.utils.DataSchema;
import org.apache.pinot.common.utils.DataSchema.ColumnDataType;
import org.apache.pinot.core.common.Operator;
import org.apache.pinot.core.data.table.Key;
import org.apache.pinot.core.data.table.Record;
import org.apache.pinot.core.data.table.SimpleIndexedTable;
import org.apache.pinot.core.operator.ExecutionStatistics;
import org.apache.pinot.core.operator.blocks.results.AggregationResultsBlock;
import org.apache.pinot.core.operator.blocks.results.BaseResultsBlock;
import org.apache.pinot.core.operator.blocks.results.GroupByResultsBlock;
import org.apache.pinot.core.operator.combine.BaseCombineOperator;
import org.apache.pinot.core.plan.CombinePlanNode;
import org.apache.pinot.core.plan.PlanNode;
import org.apache.pinot.core.query.aggregation.function.AggregationFunction;
import org.apache.pinot.core.query.aggregation.function.DistinctCountHLLAggregationFunction;
import org.apache.pinot.core.query.request.context.QueryContext;
import org.apache.pinot.core.util.GroupByUtils;
import org.apache.pinot.segment.spi.AggregationFunctionType;


/**
 * The instance-level combine on the GPU: ONE ph_query_execute over every pinned segment of the query replaces the
 * per-segment operators + GroupByCombineOperator / AggregationCombineOperator (GroupByCombineOperator.java:75-252).
 * The result block is the one the stock combine returns: AggregationResultsBlock(functions, intermediate results)
 * or GroupByResultsBlock(IndexedTable, ctx) (GroupByCombineOperator.mergeResults :247), so InstanceResponseOperator,
 * DataTable serialisation and the broker reduce are unchanged.  PH_ERR_UNSUPPORTED at execution falls back to the
 * stock combine over the same segment plans.
 */
public class GpuCombinePlanNode extends CombinePlanNode {
  private final long _ctx;
  private final GpuQuery _query;
  private final GpuSegmentRegistry.Lease _segments;  // released when the launch is done
  private final List<PlanNode> _segmentPlans;
  private final QueryContext _queryContext;
  private final ExecutorService _executorService;

  public GpuCombinePlanNode(long ctx, GpuQuery query, GpuSegmentRegistry.Lease segments, List<PlanNode> segmentPlans,
      QueryContext queryContext, ExecutorService executorService) {
    super(segmentPlans, queryContext, executorService, null);
    _ctx = ctx;
    _query = query;
    _segments = segments;
    _segmentPlans = segmentPlans;
    _queryContext = queryContext;
    _executorService = executorService;
  }

  @Override
  public BaseCombineOperator run() {
    return new GpuCombineOperator();
  }

  private final class GpuCombineOperator extends BaseCombineOperator<BaseResultsBlock> {
    private final long[] _stats = new long[7];

    GpuCombineOperator() {
      super(null, Collections.emptyList(), _queryContext, _executorService);
    }

    @Override
    protected BaseResultsBlock getNextBlock() {
      long res;
      try {
        res = PinotHipJni.queryExecute(_ctx, _query._descriptor, _query._strings, _query._numGroupsLimit,
            _query._endTimeMs, _segments.handles());
      } catch (UnsupportedOperationException e) {
        return new CombinePlanNode(_segmentPlans, _queryContext, _executorService, null).run().nextBlock();
      } finally {
        _segments.close();  // the result lives in host memory: the segments may be unpinned from here on
      }
      try {
        PinotHipJni.resultStats(res, _stats);
        return _queryContext.getGroupByExpressions() == null ? aggregationBlock(res) : groupByBlock(res);
      } finally {
        PinotHipJni.resultDestroy(res);
      }
    }

    // intermediate results as the CPU functions produce them: COUNT Long, SUM / MIN / MAX Double, HLL HyperLogLog
    private Object intermediate(AggregationFunction f, ByteBuffer col, int row) {
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

    private ByteBuffer aggColumn(long res, int k, AggregationFunction f) {
      int bytes = f.getType() == AggregationFunctionType.DISTINCTCOUNTHLL
          ? 1 << ((DistinctCountHLLAggregationFunction) f).getLog2m() : 8;
      return PinotHipJni.resultAggregationBuffer(res, k, bytes).order(ByteOrder.nativeOrder());
    }

    private BaseResultsBlock aggregationBlock(long res) {
      AggregationFunction[] functions = _queryContext.getAggregationFunctions();
      List<Object> results = new ArrayList<>(functions.length);
      for (int k = 0; k < functions.length; k++) {
        results.add(intermediate(functions[k], aggColumn(res, k, functions[k]), 0));
      }
      return new AggregationResultsBlock(functions, results, _queryContext);
    }

    private BaseResultsBlock groupByBlock(long res) {
      List<ExpressionContext> groupBy = _queryContext.getGroupByExpressions();
      AggregationFunction[] functions = _queryContext.getAggregationFunctions();
      int nk = groupBy.size();
      int n = (int) PinotHipJni.resultNumGroups(res);
      String[] names = new String[nk + functions.length];
      ColumnDataType[] types = new ColumnDataType[nk + functions.length];
      ByteBuffer[] keys = new ByteBuffer[nk];
      int[] keyType = new int[nk];
      int[] keySize = new int[nk];
      for (int g = 0; g < nk; g++) {
        names[g] = groupBy.get(g).toString();
        keyType[g] = PinotHipJni.resultKeyType(res, g);
        keySize[g] = PinotHipJni.resultKeyEntrySize(res, g);
        keys[g] = PinotHipJni.resultKeyBuffer(res, g).order(ByteOrder.nativeOrder());
        types[g] = keyType[g] == PinotHipJni.INT ? ColumnDataType.INT : keyType[g] == PinotHipJni.LONG ? ColumnDataType.LONG
            : keyType[g] == PinotHipJni.FLOAT ? ColumnDataType.FLOAT : keyType[g] == PinotHipJni.DOUBLE ? ColumnDataType.DOUBLE
            : ColumnDataType.STRING;
      }
      ByteBuffer[] aggs = new ByteBuffer[functions.length];
      for (int k = 0; k < functions.length; k++) {
        names[nk + k] = functions[k].getResultColumnName();
        types[nk + k] = functions[k].getIntermediateResultColumnType();
        aggs[k] = aggColumn(res, k, functions[k]);
      }
      DataSchema schema = new DataSchema(names, types);
      // the server-level table of GroupByCombineOperator (resultSize / trim as IndexedTable.java:63-91)
      int limit = _queryContext.getLimit();
      int trimSize = GroupByUtils.getTableCapacity(limit, _queryContext.getMinServerGroupTrimSize());
      SimpleIndexedTable table = new SimpleIndexedTable(schema, _queryContext, trimSize, trimSize,
          _queryContext.getGroupTrimThreshold());
      for (int r = 0; r < n; r++) {
        Object[] kv = new Object[nk];
        Object[] row = new Object[nk + functions.length];
        for (int g = 0; g < nk; g++) {
          ByteBuffer b = keys[g];
          Object v;
          switch (keyType[g]) {
            case PinotHipJni.INT: v = b.getInt(4 * r); break;
            case PinotHipJni.LONG: v = b.getLong(8 * r); break;
            case PinotHipJni.FLOAT: v = b.getFloat(4 * r); break;
            case PinotHipJni.DOUBLE: v = b.getDouble(8 * r); break;
            default: {
              byte[] s = new byte[keySize[g]];
              b.position(r * keySize[g]);
              b.get(s);
              int len = 0;
              while (len < s.length && s[len] != 0) {
                len++;
              }
              v = new String(s, 0, len, StandardCharsets.UTF_8);
            }
          }
          kv[g] = v;
          row[g] = v;
        }
        for (int k = 0; k < functions.length; k++) {
          row[nk + k] = intermediate(functions[k], aggs[k], r);
        }
        table.upsert(new Key(kv), new Record(row));
      }
      table.finish(false);
      GroupByResultsBlock block = new GroupByResultsBlock(table, _queryContext);
      block.setNumGroupsLimitReached(_stats[6] != 0);
      return block;
    }

    @Override
    public ExecutionStatistics getExecutionStatistics() {
      // numDocsScanned, numEntriesScannedInFilter, numEntriesScannedPostFilter, numTotalDocs (SURVEY 8(a26))
      return new ExecutionStatistics(_stats[0], _stats[1], _stats[2], _stats[3]);
    }

    @Override
    protected void processSegments() {
    }

    @Override
    protected void onProcessSegmentsException(Throwable t) {
    }

    @Override
    protected void onProcessSegmentsFinish() {
    }

    @Override
    public List<Operator> getChildOperators() {
      return Collections.emptyList();
    }

    @Override
    public String toExplainString() {
      return "COMBINE_GPU";
    }
  }
}
