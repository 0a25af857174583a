package org.apache.pinot.core.gpu;

import java.util.List;
import org.apache.pinot.common.request.context.ExpressionContext;
import org.apache.pinot.common.utils.DataSchema;
import org.apache.pinot.common.utils.DataSchema.ColumnDataType;
import org.apache.pinot.core.query.aggregation.function.AggregationFunction;
import org.apache.pinot.core.query.request.context.QueryContext;


/**
 * The DataSchema of a GPU group-by result, as GroupByOperator builds it (GroupByOperator.java:66-86): the group-by
 * expressions with the stored types of their key columns, then each function's result column name and intermediate
 * type.
 */
final class GpuResultSchema {
  private GpuResultSchema() {
  }

  static ColumnDataType keyType(int phType) {
    switch (phType) {
      case PinotHipJni.INT: return ColumnDataType.INT;
      case PinotHipJni.LONG: return ColumnDataType.LONG;
      case PinotHipJni.FLOAT: return ColumnDataType.FLOAT;
      case PinotHipJni.DOUBLE: return ColumnDataType.DOUBLE;
      default: return ColumnDataType.STRING;
    }
  }

  static DataSchema of(QueryContext ctx, long res) {
    List<ExpressionContext> groupBy = ctx.getGroupByExpressions();
    AggregationFunction[] functions = ctx.getAggregationFunctions();
    int nk = groupBy.size();
    String[] names = new String[nk + functions.length];
    ColumnDataType[] types = new ColumnDataType[nk + functions.length];
    for (int g = 0; g < nk; g++) {
      names[g] = groupBy.get(g).toString();
      types[g] = keyType(PinotHipJni.resultKeyType(res, g));
    }
    for (int k = 0; k < functions.length; k++) {
      names[nk + k] = functions[k].getResultColumnName();
      types[nk + k] = functions[k].getIntermediateResultColumnType();
    }
    return new DataSchema(names, types);
  }
}
